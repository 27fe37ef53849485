"""Config enums, same names and values as gym_pybullet_drones/utils/enums.py:3-48."""
from enum import Enum


class DroneModel(Enum):
    """Drone models (only CF2X has a DSL PID and a DYN torque model here)."""
    CF2X = "cf2x"
    CF2P = "cf2p"
    RACE = "racer"


class Physics(Enum):
    """Physics implementations.

    DYN is the explicit dynamics model (BaseAviary._dynamics, BA:815-892) and is
    what the HIP integrator implements.  The PYB_* modes are Bullet-integrated in
    the reference; here PYB_GND / PYB_DRAG / PYB_DW / PYB_GND_DRAG_DW map to DYN
    plus the corresponding force models (build-defined) and
    PYB itself is not implemented yet.
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
