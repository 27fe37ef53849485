"""MI355X-native quadrotor-swarm step (HIP) + on-device MAPPO.

Drop-in for the per-control-step hot path of khuzema-h/marl-gym-pybullet-drones
(gym_pybullet_drones): envs (MultiHoverAviary / SpiralFormationAviary), the
baselines VecEnv surface, and the mappo trainer API.  See DESIGN.md.
"""
from .utils.enums import DroneModel, Physics, ImageType, ActionType, ObservationType

__version__ = "0.1.0"
__all__ = ["DroneModel", "Physics", "ImageType", "ActionType", "ObservationType"]
