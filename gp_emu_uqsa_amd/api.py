"""Public API with the reference's signatures (emulatorfunctions.py:13-286):
setup, train, plot, posterior, posterior_sample."""
from __future__ import annotations

import numpy as _np

from . import files as _files
from . import kernels as _kernels
from . import model as _model
from . import native as _native
from . import optimize as _optimize
from . import plotting as _plotting


def setup(config_file, datashuffle=True, scaleinputs=True):
    """Read config + beliefs, load and split the data, build kernel, data sets,
    validation posterior and optimiser; return an Emulator (reference :13-57)."""
    config = _files.Config(config_file)
    beliefs = _files.Beliefs(config.beliefs)
    par = _model.Hyperparams(beliefs)
    basis = _model.Basis(beliefs)
    tv_conf = _model.TV_config(*config.tv_config)
    all_data = _model.All_Data(config.inputs, config.outputs, tv_conf, beliefs, par,
                               datashuffle, scaleinputs)
    if beliefs.alt_nugget != "T":
        K = _kernels.kernel(all_data.x_full.shape[1], par)
    else:
        print("\n*** Using alternative nugget ***")
        K = _kernels.kernel_alt_nug(all_data.x_full.shape[1], par)
    x_T, y_T = all_data.choose_T()
    x_V, y_V = all_data.choose_V()
    training = _model.Data(x_T, y_T, basis, par, beliefs, K)
    validation = _model.Data(x_V, y_V, basis, par, beliefs, K)
    post = _model.Posterior(validation, training, par, beliefs, K)
    opt_T = _optimize.Optimize(training, basis, par, beliefs, config)
    return _model.Emulator(config, beliefs, par, basis, tv_conf, all_data, training,
                           validation, post, opt_T, K)


def train(E, auto=True, message=False, no_retrain=False):
    """Train on T, validate on V, optionally fold V into T and repeat; write the
    updated beliefs and T-data files (reference :61-124)."""
    E.tv_conf.auto_train(auto, no_retrain)
    while E.tv_conf.doing_training():
        print("\n*** Training round", E.tv_conf.no_of_trains, "***")
        print("Training points:", E.training.inputs.shape[0])
        E.opt_T.llh_optimize(message)
        E.training.remake()
        E.validation.remake()
        E.post.remake()
        E.post.mahalanobis_distance()
        E.post.indiv_standard_error(ise=2.0)
        E.beliefs.final_beliefs(E, False)
        E.post.final_design_points(E, False)
        if E.tv_conf.check_still_training():
            print("Preparing for next round of training...")
            E.post.incVinT()
            E.tv_conf.next_Vset()
            E.all_data.choose_new_V(E.validation)
            E.training.remake()
            E.validation.remake()
            E.post.remake()
    if E.tv_conf.do_final_build():
        print("\n*** Doing final build ***")
        if E.tv_conf.noV != 0 and E.training.inputs.shape[0] < E.all_data.numpoints:
            E.post.incVinT()
        E.training.remake()
        E.opt_T.llh_optimize(message)
        E.training.remake()
        E.beliefs.final_beliefs(E, True)
        E.post.final_design_points(E, True)
    return None


def _as_points(E, x):
    x = _np.asarray(x, dtype=float)
    if x[0].size == 1:
        x = _np.array([x]).T
    if x[0, :].size != E.training.inputs[0, :].size:
        print("ERROR: test points have different number of columns to data in emulator. Exiting.")
        raise SystemExit(1)
    return x


def posterior(E, x, predict=True):
    """(mean, full covariance) at x (reference :226-252)."""
    x = _as_points(E, x)
    xs = _model.Data(x, None, E.basis, E.par, E.beliefs, E.K)
    p = _model.Posterior(xs, E.training, E.par, E.beliefs, E.K, predict=predict)
    return p.mean, p.var


def posterior_sample(E, x, predict=True):
    """mean + chol(var) u, u ~ N(0, I) from np.random (reference :255-286); the
    Cholesky of the posterior covariance runs on the GPU (gpe_cholesky)."""
    x = _as_points(E, x)
    xs = _model.Data(x, None, E.basis, E.par, E.beliefs, E.K)
    p = _model.Posterior(xs, E.training, E.par, E.beliefs, E.K, predict=predict)
    L = _native.default_context().cholesky(p.var, want=("L",))["L"]
    u = _np.random.randn(x.shape[0])
    return p.mean + L.dot(u)


def plot(E, plot_dims, fixed_dims=[], fixed_vals=[], mean_or_var="mean", customLabels=[],
         points=False, predict=True):
    """1-D or 2-D plot of the posterior mean or variance on a 30 x 30 grid
    (reference :128-223); the variance uses the diagonal-only posterior path."""
    return _plotting.plot(E, plot_dims, fixed_dims, fixed_vals, mean_or_var, customLabels,
                          points, predict)
