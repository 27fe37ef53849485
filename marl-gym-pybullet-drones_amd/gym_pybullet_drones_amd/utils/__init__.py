from .enums import DroneModel, Physics, ImageType, ActionType, ObservationType
from .spaces import Box

__all__ = ["DroneModel", "Physics", "ImageType", "ActionType", "ObservationType", "Box"]
