"""Applications built on the implicit global grid: 3-D heat diffusion (the
benchmark) and 2-D staggered acoustics."""
from .acoustic2d import Acoustic2D, acoustic2d_reference  # noqa: F401
from .diffusion3d import Diffusion3D, run_diffusion3d, t_eff_gbs  # noqa: F401
