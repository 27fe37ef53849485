'''MAPPO controller package (gym_pybullet_drones/mappo/__init__.py:3-16), on-device.'''

from .config import MAPPO_CONFIG


def __getattr__(name):   # keep `import ...mappo` light (torch models load on first use)
    if name == 'MAPPO':
        from .mappo import MAPPO
        return MAPPO
    if name in ('MAPPOAgent', 'MAPPOActorCritic', 'MLPActor'):
        from . import agent
        return getattr(agent, name)
    if name in ('MAPPOBuffer', 'compute_returns_and_advantages', 'normalize_advantages'):
        from . import buffer
        return getattr(buffer, name)
    if name in ('normalize_tensor', 'explained_variance'):
        from . import utils
        return getattr(utils, name)
    raise AttributeError(name)


__all__ = ['MAPPO', 'MAPPOAgent', 'MAPPOActorCritic', 'MLPActor', 'MAPPOBuffer', 'compute_returns_and_advantages',
           'normalize_advantages', 'MAPPO_CONFIG', 'normalize_tensor', 'explained_variance']
