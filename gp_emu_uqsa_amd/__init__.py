"""gp_emu_uqsa_amd -- MI355X-native hot path of the GP_emu_UQSA Gaussian-process
emulator, behind the reference's API:

    import gp_emu_uqsa_amd as g
    E = g.setup("toy-sim_config")
    g.train(E)
    mean, var = g.posterior(E, x)

The covariance build, Cholesky factorisation, triangular solves, log-marginal-
likelihood gradient and posterior run in libgpemu.so (hand-written HIP for
gfx950, C-ABI in include/gpemu.h); there is no CPU fallback.
"""
from .api import plot, posterior, posterior_sample, setup, train  # noqa: F401

__all__ = ["setup", "train", "plot", "posterior", "posterior_sample"]
__version__ = "0.1.0"
