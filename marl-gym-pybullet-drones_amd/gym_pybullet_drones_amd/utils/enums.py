"""Config enums, same names and values as gym_pybullet_drones/utils/enums.py:3-48."""
from enum import Enum


class DroneModel(Enum):
    """Drone models (CF2X and CF2P: the two with a DSL PID, DSLPIDControl.py:34-36)."""
    CF2X = "cf2x"
    CF2P = "cf2p"
    RACE = "racer"


class Physics(Enum):
    """Physics implementations.

    DYN is the explicit dynamics model (BaseAviary._dynamics, BA:815-892).  PYB
    and PYB_GND / PYB_DRAG / PYB_DW / PYB_GND_DRAG_DW are the kernel's
    restatement of Bullet's step of the _physics forces (plus the named force
    models); DYN plus force models is available through
    QuadSwarm(aux=...) (build-defined, SURVEY §8 physics-mode note).
    """
    PYB = "pyb"
    DYN = "dyn"
    PYB_GND = "pyb_gnd"
    PYB_DRAG = "pyb_drag"
    PYB_DW = "pyb_dw"
    PYB_GND_DRAG_DW = "pyb_gnd_drag_dw"


class ImageType(Enum):
    RGB = 0
    DEP = 1
    SEG = 2
    BW = 3


class ActionType(Enum):
    RPM = "rpm"
    PID = "pid"
    VEL = "vel"
    ONE_D_RPM = "one_d_rpm"
    ONE_D_PID = "one_d_pid"


class ObservationType(Enum):
    KIN = "kin"
    RGB = "rgb"
