"""Heteroscedastic noise fitting.

Mirrors gp_emu_uqsa.noise_fit (noise_fit/noise_fit.py:38-228): `noisefit(data, noise,
stopat, olhcmult, samples, fileStr)` keeps the reference's checks and messages, its
np.random consumption (setup's shuffles, train's guesses, then per estimation step
`samples` successive randn draws of the set's size, then the final oLHC design), the
'zp-outputs' file it rewrites each iteration, and the 'x_range_input',
'noise-inputs' and 'noise-outputs' files.

The estimation step (:130-150) is where the reference spends its time outside
training: a full m x m posterior covariance, np.linalg.cholesky of it, and `samples`
matrix-vector products L.dot(u) in a Python loop.  Here each step is one call of
gpe_noise_sample: the covariance is built, factored (the library's blocked Cholesky)
and multiplied by all draws at once (one MFMA GEMM) on the GPU, and only the m sums
of squared residuals come back.  The draws are the reference's:
np.random.randn(samples, m) yields, row by row, exactly the values of `samples`
successive np.random.randn(m) calls.
"""
from __future__ import annotations

import numpy as _np

from . import api as _api
from . import design_inputs as _gd
from . import model as _model
from . import native as _native


def _transform(x, reg="log"):
    """z = log(y) (:10-14)."""
    return _np.log(x) if reg == "log" else x


def _untransform(x, reg="log"):
    """y = exp(z) (:17-21)."""
    return _np.exp(x) if reg == "log" else x


def _read_file(ifile):
    """key value per line, split on the first space (:23-34)."""
    print("*** Reading file:", ifile, "***")
    dct = {}
    try:
        with open(ifile, "r") as f:
            for line in f:
                (key, val) = line.split(" ", 1)
                dct[key] = val.strip()
        return dct
    except OSError:
        print("ERROR: Problem reading file.")
        raise SystemExit(1)


def estimate_noise(E, xp, t, samples):
    """z' = log( (1/s) sum_j 0.5 (t - (mean + L u_j))^2 ), u_j ~ randn(t.size), for the
    posterior of emulator E at the points of Data xp (:130-139 and :142-150)."""
    m = int(_np.size(t))
    U = _np.random.randn(samples, m)
    if m == 0:
        return _transform(_np.zeros(0) / float(samples))
    ctx = _model.upload_training(E.training)
    ctx.ensure_factor(E.K.kind, E.K.d, float(E.K.n), 1.0, E.training.r_scale())
    rs = xp.r_scale()
    try:
        _, zsum = ctx.noise_sample(xp.inputs, xp.H, E.par.beta, float(E.par.sigma), t, U,
                                   r_new=None if rs == 0.0 else xp.r, r_scale=rs)
    except _native.NotPositiveDefinite as e:
        raise _np.linalg.LinAlgError("Matrix is not positive definite (" + str(e) + ")") from None
    return _transform(zsum / float(samples))


def noisefit(data, noise, stopat=20, olhcmult=100, samples=200, fileStr=""):
    """Fit one emulator to the mean of the data and another to its noise (:38-228).
    Results are saved to 'noise-inputs' and 'noise-outputs' (prefixed by fileStr_)."""
    datac, noisec = _read_file(data), _read_file(noise)
    datab, noiseb = _read_file(datac["beliefs"]), _read_file(noisec["beliefs"])
    if datac["inputs"] != noisec["inputs"]:
        print("\nWARNING: different inputs files in config files. Exiting.")
        return None
    if datab["alt_nugget"] == "F":
        print("\nWARNING: data beliefs must have alt_nugget T. Exiting.")
        return None
    if datab["fix_nugget"] == "T" or noiseb["fix_nugget"] == "T":
        print("\nWARNING: data and noise beliefs need fix_nugget F. Exiting.")
        return None
    if datac["tv_config"] != noisec["tv_config"]:
        print("\nWARNING: different tv_config in config files. Exiting.")
        return None
    if noisec["outputs"] != "zp-outputs":
        print("\nWARNING: config outputs file must be 'zp-outputs'. Exiting.")
        return None

    GD = _api.setup(data, datashuffle=True, scaleinputs=False)
    _np.savetxt("zp-outputs",
                _np.zeros(GD.training.outputs.size + GD.validation.outputs.size * GD.tv_conf.noV).T)
    GN = _api.setup(noise, datashuffle=True, scaleinputs=False)
    # if shuffled, fix the inconsistencies (:79-83)
    GN.training.inputs = GD.training.inputs
    GN.validation.inputs = GD.validation.inputs
    GN.training.remake()
    GN.validation.remake()

    if GD.all_data.tv.noV > 1:
        print("\nWARNING: should have 0 or 1 validation sets for noise fitting. Exiting.")
        raise SystemExit(1)
    valsets = GD.all_data.tv.noV != 0

    print("\n****************"
          "\nTRAIN GP ON DATA"
          "\n****************")
    x = GD.training.inputs
    t = GD.training.outputs
    xv = GD.validation.inputs
    tv = GD.validation.outputs
    _api.train(GD, no_retrain=valsets)

    r = _np.zeros(t.size)
    rv = _np.zeros(tv.size)
    count = 0
    while True:
        xp = _model.Data(x, None, GD.basis, GD.par, GD.beliefs, GD.K)
        xvp = _model.Data(xv, None, GD.basis, GD.par, GD.beliefs, GD.K)
        if count > 0:
            xp.set_r(r)
            xp.make_A(s2=GD.par.sigma ** 2, predict=True)
            xvp.set_r(rv)
            xvp.make_A(s2=GD.par.sigma ** 2, predict=True)
        count = count + 1

        print("\n***********************"
              "\nESTIMATING NOISE LEVELS " + str(count) +
              "\n***********************")
        z_prime = estimate_noise(GD, xp, t, samples)
        _np.savetxt("zp-outputs", z_prime)
        z_prime_V = estimate_noise(GD, xvp, tv, samples)

        print("\n*****************"
              "\nTRAIN GP ON NOISE " + str(count) +
              "\n*****************")
        GN.training.outputs = z_prime.T
        GN.training.remake()
        GN.validation.outputs = z_prime_V.T
        GN.validation.remake()
        GN.tv_conf.no_of_trains = 0
        GN.tv_conf.retrain = "y"
        _api.train(GN, no_retrain=valsets)

        print("\n***********************************"
              "\nTRAIN GP ON DATA WITH NOISE FROM GP " + str(count) +
              "\n***********************************")
        xp_GN = _model.Data(x, None, GN.basis, GN.par, GN.beliefs, GN.K)
        p_GN = _model.Posterior(xp_GN, GN.training, GN.par, GN.beliefs, GN.K, full_var=False)
        r = _untransform(p_GN.mean)
        GD.training.set_r(r)
        v_GN = _model.Data(xv, None, GN.basis, GN.par, GN.beliefs, GN.K)
        pv_GN = _model.Posterior(v_GN, GN.training, GN.par, GN.beliefs, GN.K, full_var=False)
        rv = _untransform(pv_GN.mean)
        GD.validation.set_r(rv)
        GD.tv_conf.no_of_trains = 0
        GD.tv_conf.retrain = "y"
        _api.train(GD, no_retrain=valsets)

        if count == stopat:
            print("\nCompleted", count, "fits, stopping here.")
            print("\nGenerating input points to predict noise values at...")
            n = x[0].size * int(olhcmult)
            N = int(n)
            olhc_range = [[_np.amin(col), _np.amax(col)] for col in x.T]
            filename = "x_range_input"
            _gd.optLatinHyperCube(x[0].size, n, N, olhc_range, filename)
            x_range = _np.loadtxt(filename)
            if x[0].size == 1:
                x_range = _np.array([x_range, ]).T
            x_plot = _model.Data(x_range, None, GN.basis, GN.par, GN.beliefs, GN.K)
            p_plot = _model.Posterior(x_plot, GN.training, GN.par, GN.beliefs, GN.K, full_var=False)
            mean_plot = p_plot.mean
            p_plot.interval()
            UI, LI = p_plot.UI, p_plot.LI
            print("\nSaving results to file...")
            nfileStr = fileStr + "_" if fileStr != "" else fileStr
            _np.savetxt(nfileStr + "noise-inputs", x_range)
            _np.savetxt(nfileStr + "noise-outputs", _np.transpose(
                [_np.sqrt(_untransform(mean_plot)),
                 _np.sqrt(_untransform(LI)), _np.sqrt(_untransform(UI))]))
            break
    return None
