from .swarm import QuadSwarm, StepResult, grid_layout
from .aviaries import MultiHoverAviary, SpiralFormationAviary

__all__ = ["QuadSwarm", "StepResult", "grid_layout", "MultiHoverAviary", "SpiralFormationAviary"]
