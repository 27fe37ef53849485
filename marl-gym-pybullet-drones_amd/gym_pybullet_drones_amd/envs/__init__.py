from .swarm import QuadSwarm, StepResult, grid_layout
from .aviaries import (FlockAviary, LeaderFollowerAviary, MeetupAviary, MultiHoverAviary,
                       SpiralFormationAviary)

__all__ = ["QuadSwarm", "StepResult", "grid_layout", "MultiHoverAviary", "SpiralFormationAviary", "FlockAviary",
           "MeetupAviary", "LeaderFollowerAviary"]
