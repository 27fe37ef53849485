"""MAPPO default configuration — same keys and defaults as gym_pybullet_drones/mappo/config.py:3-49.

Extra keys (all optional, build-specific):
  use_graphs      capture the rollout step and the update iteration as HIP graphs
  reference_compat reproduce reference quirks (double obs normalisation on done, MP:804/1037)
  precision       4 (fp32) or 8 (fp64) simulator state
  initial_xyzs    explicit drone layout (required for MultiHover with >= 6 drones, SURVEY §7 hard-2)
"""

MAPPO_CONFIG = {
    # Model args
    'hidden_dim': 64,
    'activation': 'tanh',
    'norm_obs': False,
    'norm_reward': False,
    'clip_obs': 10,
    'clip_reward': 10,

    # MAPPO-specific args
    'share_actor_weights': True,
    'centralized_critic': True,
    'include_actions_in_critic': False,
    'global_state_dim': None,

    # Loss args
    'gamma': 0.99,
    'use_gae': True,
    'gae_lambda': 0.95,
    'use_clipped_value': False,
    'clip_param': 0.2,
    'target_kl': 0.01,
    'entropy_coef': 0.01,

    # Optim args
    'opt_epochs': 10,
    'mini_batch_size': 64,
    'actor_lr': 0.0003,
    'critic_lr': 0.001,
    'max_grad_norm': 0.5,   # configured but never applied by the reference; same here

    # Runner args
    'max_env_steps': 1000000,
    'num_workers': 16,      # accepted for compatibility; there is no worker pool (envs run on the GPU)
    'rollout_batch_size': 4,
    'rollout_steps': 100,
    'deque_size': 10,
    'eval_batch_size': 10,

    # Misc
    'log_interval': 1000,
    'save_interval': 50000,
    'num_checkpoints': 5,
    'eval_interval': 10000,
    'eval_save_best': True,
    'tensorboard': True,    # accepted; logging here is stdout + CSV (observability is out of scope)
}
