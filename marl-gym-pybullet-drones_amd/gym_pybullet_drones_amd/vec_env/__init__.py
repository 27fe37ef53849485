from .vec_env import (VecEnv, VecEnvWrapper, SwarmVecEnv, VecRecordEpisodeStatistics, observation_space_for,
                      action_space_for)

__all__ = ["VecEnv", "VecEnvWrapper", "SwarmVecEnv", "VecRecordEpisodeStatistics", "observation_space_for",
           "action_space_for"]
