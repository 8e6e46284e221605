"""Generate golden vectors by running the REFERENCE (GP_emu_UQSA) in the build
container.  The reference never travels: only the .npz outputs are committed.

Run from the repo root:  python tests/golden/make_golden.py [G1 G2 G3 G4 G5]

Fixtures:
  G1 kernel_*.npz      K.var / covar / grad_delta_A / grad_nugget_A, both kernels
  G2 objective_*.npz   loglikelihood_gp4ml / _mucm (LLH, grad) incl. a non-PD case
  G3 posterior_*.npz   reconstructed example emulators: posterior mean/var, beta
  G4 train_*.npz       seeded toy-sim g.train() trajectory (objective x's, result)
  G5 scale_4096.npz    n=4096 d=10 gp4ml LLH+grad (X regenerated from the seed)
  G6 host_*.npz        host-side setup() state: shuffle, T/V split, H, bounds, RNG
  G7 history_match.npz imp_plot IMP/ODP grids + oLHC designs, nonimp_data, new_wave_design
  G8 sensitivity_*.npz uncertainty / sensitivity / main + interaction effects / total-effect
                       variance (case2) on the reconstructed toysim3D emulators and on a
                       synthetic untrained n=300, d=4 emulator, with the intermediates
  G9 noise_fit.npz     seeded noisefit() on a 2-D heteroscedastic data set (n=60): every
                       posterior and Cholesky of the noise loop, the randn draws, each
                       z' written to zp-outputs, the final noise-inputs/-outputs and beliefs
Versions of numpy/scipy used are stored in every file ("meta").
"""
from __future__ import annotations

import contextlib
import io
import json
import os
import shutil
import sys
import tempfile
import time
import types

import numpy as np
import scipy

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
REF = "/root/reference"
sys.path.insert(0, REF)
sys.path.insert(0, REPO)
os.environ.setdefault("MPLBACKEND", "Agg")

with contextlib.redirect_stdout(io.StringIO()):
    import gp_emu_uqsa as g                              # noqa: E402
    import gp_emu_uqsa._emulatorkernels as emuk          # noqa: E402
    import gp_emu_uqsa._emulatorclasses as emuc          # noqa: E402
    import gp_emu_uqsa._emulatoroptimise as emuo         # noqa: E402

from oracle import gp_oracle as orc                      # noqa: E402  (synthetic data only)

META = json.dumps({"numpy": np.__version__, "scipy": scipy.__version__,
                   "reference": "GP_emu_UQSA @ /root/reference",
                   "generated": time.strftime("%Y-%m-%d")})


def save(name, **arrays):
    path = os.path.join(HERE, name)
    np.savez_compressed(path, meta=np.array(META), **arrays)
    print("wrote", path, {k: np.shape(v) for k, v in arrays.items()})


def quiet(fn, *a, **k):
    with contextlib.redirect_stdout(io.StringIO()):
        return fn(*a, **k)


# ---------------------------------------------------------------- helpers
def ref_kernel(kind, delta, nu):
    par = types.SimpleNamespace(delta=np.array(delta, float), nugget=nu)
    cls = emuk.kernel_alt_nug if kind == orc.ALT else emuk.kernel
    return cls(len(delta), par)


def ref_data(X, f, kind, delta, nu, r=None):
    """A real reference Data object with a linear basis 1, x_0..x_{d-1}."""
    d = X.shape[1]
    basis = types.SimpleNamespace(h=[lambda x: 1.0] + [lambda x: x] * d,
                                  basis_inf=list(range(d)))
    beliefs = types.SimpleNamespace(alt_nugget="T" if kind == orc.ALT else "F")
    par = types.SimpleNamespace(beta=np.zeros(d + 1), delta=np.array(delta, float),
                                nugget=nu, sigma=1.0)
    K = ref_kernel(kind, delta, nu)
    data = emuc.Data(X.copy(), f.copy(), basis, par, beliefs, K)
    if r is not None:
        data.set_r(np.asarray(r, float), message=False)
    return data, par


def ref_objective(X, f, kind, variant, fit_nugget, hp, nu_fixed, r=None):
    d = X.shape[1]
    delta = list(hp[:d])
    nu = hp[d] if fit_nugget else nu_fixed
    data, par = ref_data(X, f, kind, delta, nu, r)
    self = types.SimpleNamespace(data=data, par=par)
    x = 2.0 * np.log(np.asarray(hp, float))
    fn = emuo.Optimize.loglikelihood_gp4ml if variant == orc.GP4ML else \
        emuo.Optimize.loglikelihood_mucm
    out = quiet(fn, self, x)
    if out is None:
        return None
    llh, grad = out
    sig2 = par.sigma ** 2
    return float(llh), np.array(grad, float), float(sig2), data.H.copy()


# ---------------------------------------------------------------- G1
def make_g1():
    rs = np.random.RandomState(11)
    X = rs.uniform(size=(64, 3))
    Xs = rs.uniform(size=(16, 3))
    delta = np.array([0.7, 0.35, 1.3])
    for kind, tag in ((orc.STD, "std"), (orc.ALT, "alt")):
        nu = 0.05
        K = ref_kernel(kind, delta, nu)
        A_pred = K.var(X, True).copy()
        A_est = K.var(X, False).copy()
        e = K.exp_save.copy()
        gd = np.stack([K.grad_delta_A(X[:, i], i, 1.7) for i in range(3)])
        gn = K.grad_nugget_A(X, 1.7)
        cov = K.covar(X, Xs)
        save(f"kernel_{tag}.npz", X=X, Xs=Xs, delta=delta, nu=nu, s2=1.7,
             A_pred=A_pred, A_est=A_est, exp_save=e, grad_delta=gd,
             grad_nugget=gn, covar=cov)


# ---------------------------------------------------------------- G2
G2_CASES = [
    # (tag, kind, variant, fit_nugget, use_r)
    ("std_gp4ml_fitnug", orc.STD, orc.GP4ML, True, False),
    ("std_gp4ml_fixnug", orc.STD, orc.GP4ML, False, False),
    ("std_mucm_fitnug", orc.STD, orc.MUCM, True, False),
    ("std_mucm_fixnug", orc.STD, orc.MUCM, False, False),
    ("alt_gp4ml_fitnug", orc.ALT, orc.GP4ML, True, False),
    ("alt_gp4ml_fixnug", orc.ALT, orc.GP4ML, False, False),
    ("alt_gp4ml_fitnug_r", orc.ALT, orc.GP4ML, True, True),
    # std kernel with Data.set_r: A carries no r, the sigma gradient subtracts it
    ("std_gp4ml_fitnug_r", orc.STD, orc.GP4ML, True, True),
    ("std_gp4ml_fixnug_r", orc.STD, orc.GP4ML, False, True),
]


def g2_hp(d, variant, fit_nugget, delta, nu, sigma):
    hp = list(np.full(d, delta) if np.isscalar(delta) else delta)
    if fit_nugget:
        hp.append(nu)
    if variant == orc.GP4ML:
        hp.append(sigma)
    return np.array(hp, float)


def make_g2():
    for (n, d) in ((200, 3), (1024, 10)):
        X, f, _ = orc.synthetic_problem(n, d, seed=3)
        rs = np.random.RandomState(5)
        r = 0.01 * rs.uniform(size=n)
        out = {"X": X, "f": f, "r": r}
        points = [(1.0, 1e-3, 1.0), (np.linspace(0.3, 1.2, d), 2e-2, 0.7)]
        for tag, kind, variant, fitn, use_r in G2_CASES:
            for pi, (delta, nu, sigma) in enumerate(points):
                hp = g2_hp(d, variant, fitn, delta, nu, sigma)
                t0 = time.time()
                res = ref_objective(X, f, kind, variant, fitn, hp, nu, r if use_r else None)
                key = f"{tag}_p{pi}"
                out[key + "_hp"] = hp
                out[key + "_nufixed"] = np.array(nu)
                out[key + "_llh"] = np.array(res[0])
                out[key + "_grad"] = res[1]
                out[key + "_sig2"] = np.array(res[2])
                print(f"  n={n} {key} llh={res[0]:.10g} ({time.time()-t0:.1f}s)")
        # non-PD: huge length scales, zero nugget -> numerically singular A
        hp = g2_hp(d, orc.GP4ML, False, 200.0, 0.0, 1.0)
        res = ref_objective(X, f, orc.STD, orc.GP4ML, False, hp, 0.0)
        assert res is None, "expected the reference to report non-PD"
        out["nonpd_hp"] = hp
        save(f"objective_n{n}_d{d}.npz", **out)


# ---------------------------------------------------------------- G3
RECON = [
    ("toysim", "examples/toy-sim/reconstruct", "toy-sim_config_recon", 2),
    ("toysim3d_o0", "examples/sensitivity_multi_outputs/sensitivity_recon",
     "toysim3D_config0_recon", 3),
    ("toysim3d_o1", "examples/sensitivity_multi_outputs/sensitivity_recon",
     "toysim3D_config1_recon", 3),
]


def make_g3():
    for tag, sub, conf, d in RECON:
        tmp = tempfile.mkdtemp()
        shutil.copytree(os.path.join(REF, sub), os.path.join(tmp, "w"))
        cwd = os.getcwd()
        os.chdir(os.path.join(tmp, "w"))
        try:
            E = quiet(g.setup, conf, datashuffle=False, scaleinputs=True)
            rs = np.random.RandomState(17)
            xs = rs.uniform(size=(20, d))
            mean, var = quiet(g.posterior, E, xs)
            # a14, before optimalbeta changes E.par.beta: seeded posterior_sample
            # (emulatorfunctions.py:255-286), and on a validation-style set (outputs
            # drawn around the posterior, some >= 2 sd away) interval /
            # indiv_standard_error / mahalanobis_distance (_emulatorclasses.py:635-676)
            np.random.seed(23)
            sample = quiet(g.posterior_sample, E, xs)
            rs2 = np.random.RandomState(29)
            ys = mean + rs2.normal(scale=1.5, size=mean.size) * np.sqrt(np.abs(np.diag(var)))
            Dv = emuc.Data(xs.copy(), ys.copy(), E.basis, E.par, E.beliefs, E.K)
            p = quiet(emuc.Posterior, Dv, E.training, E.par, E.beliefs, E.K)
            p.interval()
            buf = io.StringIO()
            with contextlib.redirect_stdout(buf):
                ise_retrain = p.indiv_standard_error(ise=2.0)
            ise_text = buf.getvalue()
            buf = io.StringIO()
            with contextlib.redirect_stdout(buf):
                p.mahalanobis_distance()
            md_text = buf.getvalue()
            md = float(md_text.split("calculated Mahalanobis_distance:")[1].split()[0])
            beta_stored = E.par.beta.copy()
            A = E.training.A.copy()
            quiet(E.opt_T.optimalbeta)
            beta_opt = E.par.beta.copy()
            out = dict(XT=E.training.inputs, fT=E.training.outputs, HT=E.training.H,
                       xs=xs, mean=mean, var=var, A_trace=np.trace(A), A_sum=A.sum(),
                       sample_seed=np.array(23), sample=sample, ys=ys, LI=p.LI, UI=p.UI,
                       ise_retrain=np.array(ise_retrain), ise_text=np.array(ise_text),
                       md=np.array(md), md_text=np.array(md_text),
                       beta=beta_stored, beta_opt=beta_opt,
                       delta=np.array(E.par.delta, float), nu=np.array(E.par.nugget),
                       sigma=np.array(E.par.sigma),
                       alt=np.array(E.beliefs.alt_nugget == "T"),
                       mucm=np.array(E.beliefs.mucm == "T"),
                       fix_nugget=np.array(E.beliefs.fix_nugget == "T"))
            save(f"posterior_{tag}.npz", **out)
        finally:
            os.chdir(cwd)
            shutil.rmtree(tmp)


# ---------------------------------------------------------------- G4
def make_g4():
    for seed in (0, 1):
        tmp = tempfile.mkdtemp()
        shutil.copytree(os.path.join(REF, "examples/toy-sim"), os.path.join(tmp, "w"))
        cwd = os.getcwd()
        os.chdir(os.path.join(tmp, "w"))
        try:
            np.random.seed(seed)
            E = quiet(g.setup, "toy-sim_config")
            calls = []
            orig = E.opt_T.loglikelihood_mucm

            def rec(x, _orig=orig):
                res = _orig(x)
                calls.append((np.array(x, float), None if res is None else res[0]))
                return res
            E.opt_T.loglikelihood_mucm = rec
            log = io.StringIO()
            with contextlib.redirect_stdout(log):
                g.train(E, auto=True)
            xs = np.array([c[0] for c in calls])
            ll = np.array([np.nan if c[1] is None else c[1] for c in calls])
            beliefs = {}
            for fn in sorted(os.listdir(".")):
                if fn.startswith("toy-sim_beliefs-"):
                    beliefs[fn] = open(fn).read()
            rs = np.random.RandomState(23)
            xs_post = rs.uniform(size=(10, 2))
            pm, pv = quiet(g.posterior, E, xs_post)
            save(f"train_toysim_seed{seed}.npz", call_x=xs, call_llh=ll,
                 delta=np.array(E.par.delta, float), sigma=np.array(E.par.sigma),
                 nugget=np.array(E.par.nugget), beta=np.array(E.par.beta, float),
                 n_train=np.array(E.training.inputs.shape[0]),
                 beliefs_json=np.array(json.dumps(beliefs)),
                 xs_post=xs_post, post_mean=pm, post_var=pv,
                 log=np.array(log.getvalue()))
        finally:
            os.chdir(cwd)
            shutil.rmtree(tmp)


# ---------------------------------------------------------------- G6 (host logic)
def make_g6():
    """Host-side state of setup(): shuffled data, T/V split, H, bounds, guess grid."""
    tmp = tempfile.mkdtemp()
    shutil.copytree(os.path.join(REF, "examples/toy-sim"), os.path.join(tmp, "w"))
    cwd = os.getcwd()
    os.chdir(os.path.join(tmp, "w"))
    try:
        np.random.seed(0)
        E = quiet(g.setup, "toy-sim_config")
        guess = np.random.random_sample(10)
        save("host_toysim_seed0.npz", x_full=E.all_data.x_full, y_full=E.all_data.y_full,
             minmax=E.all_data.minmax, XT=E.training.inputs, fT=E.training.outputs,
             HT=E.training.H, XV=E.validation.inputs, bounds=np.array(E.config.bounds, float),
             cons=np.array([[np.nan if v is None else v for v in c] for c in E.opt_T.cons], float),
             next_random=guess)
    finally:
        os.chdir(cwd)
        shutil.rmtree(tmp)


# ---------------------------------------------------------------- G5
def make_g5():
    n, d = 4096, 10
    X, f, _ = orc.synthetic_problem(n, d, seed=0)
    hp = g2_hp(d, orc.GP4ML, True, 1.0, 1e-3, 1.0)
    t0 = time.time()
    res = ref_objective(X, f, orc.STD, orc.GP4ML, True, hp, 1e-3)
    dt = time.time() - t0
    print(f"  G5 llh={res[0]:.12g} in {dt:.1f}s")
    save("scale_4096.npz", seed=np.array(0), n=np.array(n), d=np.array(d), hp=hp,
         X_sum=X.sum(), X_sq=(X ** 2).sum(), f_sum=f.sum(), llh=np.array(res[0]),
         grad=res[1], seconds=np.array(dt))


# ---------------------------------------------------------------- G7
def make_g7():
    """History matching on the reconstructed toysim3D emulators:
    imp_plot (grid 4, olhcmult 20, maxno 2), nonimp_data and new_wave_design with
    fixed seeds.  design_inputs.py:55 uses np.int, removed in NumPy 1.24: the alias
    is restored for this run (the reference's algorithm is unchanged)."""
    np.int = int
    with contextlib.redirect_stdout(io.StringIO()):
        import gp_emu_uqsa.history_match as hm
    tmp = tempfile.mkdtemp()
    shutil.copytree(os.path.join(REF, "examples/sensitivity_multi_outputs/sensitivity_recon"),
                    os.path.join(tmp, "w"))
    cwd = os.getcwd()
    os.chdir(os.path.join(tmp, "w"))
    try:
        # the example's final beliefs predate the 'active_index' line that the reference's
        # final_beliefs writes (_emulatorclasses.py:233) and that emulsetup needs
        for i in range(2):
            with open(f"toysim3D_beliefs{i}-1f", "a") as fh:
                fh.write("active_index 0 1 2\n")
        emuls = [quiet(g.setup, f"toysim3D_config{i}_recon", datashuffle=False, scaleinputs=True)
                 for i in range(2)]
        ys = [np.loadtxt(f"toysim3D_output-o{i}-1f") for i in range(2)]
        zs = [float(np.median(y)) for y in ys]
        ve = [float(0.05 * np.var(y)) for y in ys]
        out = {"zs": np.array(zs), "var_extra": np.array(ve), "cm": np.array(3.0)}
        np.random.seed(21)
        quiet(hm.imp_plot, emuls, zs, 3.0, ve, maxno=2, olhcmult=20, grid=4, plot=False)
        for s in ([0, 1], [0, 2], [1, 2]):
            tag = f"{s[0]}_{s[1]}"
            out["design_" + tag] = np.loadtxt("imp_input_" + tag)
            for m in (1, 2):
                out[f"IMP{m}_" + tag] = np.loadtxt(f"{m}_IMP_" + tag)
                out[f"ODP{m}_" + tag] = np.loadtxt(f"{m}_ODP_" + tag)
        # the example's simulator data (original units, two output columns)
        for f in ("toysim3D_input", "toysim3D_output"):
            shutil.copy(os.path.join(REF, "examples/sensitivity_multi_outputs", f), f)
        din, dout = "toysim3D_input", "toysim3D_output"
        out["data_in"] = np.loadtxt(din)
        out["data_out"] = np.loadtxt(dout)
        out["nonimp_count"] = np.array(quiet(hm.nonimp_data, emuls, zs, 3.0, ve, [din, dout], maxno=1))
        out["nonimp_in"] = np.loadtxt("nonimp_" + din)
        out["nonimp_out"] = np.loadtxt("noninp_" + dout)
        np.random.seed(22)
        out["wave_count"] = np.array(quiet(hm.new_wave_design, emuls, zs, 3.0, ve,
                                           ["nonimp_" + din, "noninp_" + dout], maxno=1, olhcmult=10))
        out["wave_design"] = np.loadtxt("nonimp_" + din)
        out["wave_olhc"] = np.loadtxt("olhc_des")
        save("history_match.npz", **out)
    finally:
        os.chdir(cwd)
        shutil.rmtree(tmp)


SENSE_ATTRS = ("uE", "uV", "uEV", "I1", "I2", "U", "U2", "S", "Stild", "Rh", "Rhh", "Rt", "Rht", "Rtt",
               "Ut", "Uht", "Utt", "Uh", "Uhh", "T", "R", "Q", "e", "W", "G")


def _sense_record(sens, m, v, tag, out):
    """Run the reference's case2 routines as its example does and keep every result."""
    quiet(sens.uncertainty)
    quiet(sens.sensitivity)
    quiet(sens.main_effect, plot=False, points=100)
    out[tag + "effect100"] = np.array(sens.effect)
    out[tag + "mean_effect100"] = np.array(sens.mean_effect)
    sens.to_file("sense_out")
    out[tag + "to_file"] = np.array(open("sense_out").read())
    quiet(sens.interaction_effect, 0, 1)
    out[tag + "interaction"] = np.array(sens.interaction)
    out[tag + "effect25"] = np.array(sens.effect)
    out[tag + "mean_effect25"] = np.array(sens.mean_effect)
    quiet(sens.totaleffectvariance)
    for a in SENSE_ATTRS:
        val = np.array(getattr(sens, a), dtype=float)
        if a == "Utt":                 # rank one (Ufact2 h h^T): one row pins it
            val = val[0]
        if a == "Rtt" and val.shape[0] > 100:   # the 90 x 90 cases pin it; keep the file small
            continue
        out[tag + a] = val
    out[tag + "senseindex"] = np.array(sens.senseindex)
    out[tag + "senseindexwb"] = np.array(sens.senseindexwb)
    out[tag + "EVTw"] = np.array(sens.EVTw)
    out[tag + "m"] = np.array(m)
    out[tag + "v"] = np.array(v)
    out[tag + "x"] = np.array(sens.x)
    out[tag + "input_range"] = np.array(sens.input_range, dtype=float)
    # the emulator state the analysis reads (training outputs, H, A as held, parameters)
    out[tag + "f"] = np.array(sens.f, dtype=float)
    out[tag + "H"] = np.array(sens.H, dtype=float)
    out[tag + "A"] = np.array(sens.A, dtype=float)
    out[tag + "beta"] = np.array(sens.beta, dtype=float)
    out[tag + "sigma"] = np.array(sens.sigma, dtype=float)
    out[tag + "nugget"] = np.array(sens.nugget, dtype=float)
    out[tag + "delta"] = 1.0 / np.sqrt(np.diag(sens.C))


def make_g8():
    """Sensitivity / UQ: the reference's sensitivity_rebuild.py
    sequence on the two reconstructed toysim3D emulators (m = 0.5, v = 0.02), and on
    a synthetic emulator (n=300, d=4, linear mean, hyperparameters from its beliefs
    file, no training).  The example's stored sense_file0/1 are not used: the current
    reference does not reproduce them on the same reconstructed emulators (EE 2.4157
    here vs 2.4277 stored), so they predate it."""
    import matplotlib
    matplotlib.use("Agg")
    with contextlib.redirect_stdout(io.StringIO()):
        import gp_emu_uqsa.sensitivity as sref
    import matplotlib.pyplot as plt
    plt.show = lambda *a, **k: None
    tmp = tempfile.mkdtemp()
    shutil.copytree(os.path.join(REF, "examples/sensitivity_multi_outputs/sensitivity_recon"),
                    os.path.join(tmp, "w"))
    cwd = os.getcwd()
    os.chdir(os.path.join(tmp, "w"))
    try:
        out = {}
        for i in range(2):
            np.random.seed(0)
            emul = quiet(g.setup, f"toysim3D_config{i}_recon", datashuffle=True, scaleinputs=True)
            m, v = [0.50, 0.50, 0.50], [0.02, 0.02, 0.02]
            sens = quiet(sref.setup, emul, m, v)
            _sense_record(sens, m, v, f"o{i}_", out)
            plt.close("all")
        save("sensitivity_toysim3d.npz", **out)
        # synthetic: n=300 points in d=4, outputs from a smooth function + noise
        n, d = 300, 4
        rng = np.random.RandomState(8)
        X = rng.uniform(size=(n, d))
        f = np.sin(3.0 * X[:, 0]) + X[:, 1] ** 2 - 0.5 * X[:, 2] * X[:, 3] + 0.01 * rng.normal(size=n)
        np.savetxt("syn_input", X, fmt="%.10f")
        np.savetxt("syn_output", f.reshape(-1, 1), fmt="%.10f")
        with open("syn_config", "w") as fh:
            fh.write("beliefs syn_beliefs\ninputs syn_input\noutputs syn_output\ntv_config 10 0 0\n"
                     "delta_bounds [ ]\nnugget_bounds [ ]\nsigma_bounds [ ]\ntries 1\nconstraints bounds\n")
        with open("syn_beliefs", "w") as fh:
            fh.write("active all\noutput 0\nbasis_str 1.0 x x x x\nbasis_inf NA 0 1 2 3\n"
                     "beta 0.3 1.1 0.4 -0.2 -0.1\ndelta 0.45 0.6 0.8 0.7\nsigma 0.9\n"
                     "nugget 0.002\nfix_nugget T\nmucm F\n")
        np.random.seed(0)
        emul = quiet(g.setup, "syn_config", datashuffle=False, scaleinputs=False)
        m, v = [0.45, 0.5, 0.55, 0.5], [0.03, 0.02, 0.05, 0.04]
        sens = quiet(sref.setup, emul, m, v)
        syn = {"X": X, "f": f}
        _sense_record(sens, m, v, "", syn)
        save("sensitivity_synthetic.npz", **syn)
    finally:
        os.chdir(cwd)
        shutil.rmtree(tmp)


NOISE_DATA_CONFIG = ("beliefs beliefs-data\ninputs INPUTS\noutputs OUTPUTS\ntv_config 10 0 0\n"
                     "delta_bounds [[0.05,10.0],[0.05,10.00]]\nsigma_bounds [[0.1,3.0]]\n"
                     "nugget_bounds [[0.001,1.05]]\ntries 3\nconstraints none\n")
NOISE_NOISE_CONFIG = ("beliefs beliefs-noise\ninputs INPUTS\noutputs zp-outputs\ntv_config 10 0 0\n"
                      "delta_bounds [[0.05,1.0],[0.05,10.00]]\nsigma_bounds [[0.001,10.0]]\n"
                      "nugget_bounds [[0.0001,1.0]]\ntries 3\nconstraints bounds\n")
NOISE_BELIEFS = ("active all\noutput 0\nbasis_str 1.0\nbasis_inf NA\nbeta 1.0\ndelta 1.0 1.0\n"
                 "sigma 1.0\nnugget 0.00001\nfix_nugget F\nalt_nugget {alt}\nmucm F\n")


def noise_fit_files(n=60, seed=3):
    """The noisefit2D example's configuration (examples/noisefit2D/config-*, beliefs-*)
    on n points of its 2-D mean + heteroscedastic-noise functions (emulator.py:12-17),
    drawn from RandomState(seed) instead of an oLHC design.  Writes into the cwd."""
    rng = np.random.RandomState(seed)
    X = rng.uniform(size=(n, 2))
    y = 3.0 * X[:, 0] ** 3 + np.exp(np.cos(10.0 * X[:, 1]) * np.cos(5.0 * X[:, 0]) ** 2)
    sd = np.abs(0.5 * X[:, 1] * (np.cos(6 * X[:, 0]) ** 2 + 0.1))
    y = y + sd * rng.normal(size=n)
    np.savetxt("INPUTS", X)
    np.savetxt("OUTPUTS", y)
    with open("config-data", "w") as fh:
        fh.write(NOISE_DATA_CONFIG)
    with open("config-noise", "w") as fh:
        fh.write(NOISE_NOISE_CONFIG)
    with open("beliefs-data", "w") as fh:
        fh.write(NOISE_BELIEFS.format(alt="T"))
    with open("beliefs-noise", "w") as fh:
        fh.write(NOISE_BELIEFS.format(alt="F"))
    return X, y


def make_g9():
    """noise_fit: np.random.seed(9); noisefit('config-data',
    'config-noise', stopat=2, olhcmult=10, samples=50).  The reference is observed, not
    changed: Posterior, np.linalg.cholesky, np.random.randn and np.savetxt are wrapped
    only to record what noisefit passes through them.  design_inputs.py:55 needs the
    np.int alias (removed in NumPy 1.24), restored as in G7."""
    np.int = int
    with contextlib.redirect_stdout(io.StringIO()):
        import gp_emu_uqsa.noise_fit.noise_fit as nf
    tmp = tempfile.mkdtemp()
    os.makedirs(os.path.join(tmp, "w"))
    cwd = os.getcwd()
    os.chdir(os.path.join(tmp, "w"))
    posts, chols, draws, zps = [], [], [], []
    orig_post, orig_chol, orig_randn, orig_savetxt = (emuc.Posterior, np.linalg.cholesky,
                                                      np.random.randn, np.savetxt)

    class RecPosterior(orig_post):
        def __init__(self, Dnew, Dold, par, beliefs, K, predict=True):
            super().__init__(Dnew, Dold, par, beliefs, K, predict)
            if Dnew.outputs is None:        # the noise loop's posteriors (train's have outputs)
                posts.append(dict(xs=np.copy(Dnew.inputs), rs=np.copy(Dnew.r) * np.ones(1),
                                  As_diag=np.copy(np.diag(Dnew.A)),
                                  x=np.copy(Dold.inputs), f=np.copy(Dold.outputs),
                                  r=np.copy(Dold.r) * np.ones(1), A_diag=np.copy(np.diag(Dold.A)),
                                  delta=np.copy(par.delta), nugget=np.array(par.nugget),
                                  sigma=np.array(par.sigma), beta=np.copy(par.beta),
                                  alt=np.array(beliefs.alt_nugget == "T"),
                                  mean=np.copy(self.mean), var=np.copy(self.var)))

    def rec_chol(a):
        L = orig_chol(a)
        if posts and np.shape(a) == posts[-1]["var"].shape and np.array_equal(a, posts[-1]["var"]):
            chols.append(np.copy(L))        # the noise loop's, not the objective's
        return L

    def rec_randn(*a):
        u = orig_randn(*a)
        draws.append(np.copy(u))
        return u

    def rec_savetxt(fname, X, *a, **k):
        if fname == "zp-outputs":
            zps.append(np.copy(X))
        return orig_savetxt(fname, X, *a, **k)

    try:
        X, y = noise_fit_files()
        emuc.Posterior, np.linalg.cholesky, np.random.randn, np.savetxt = (
            RecPosterior, rec_chol, rec_randn, rec_savetxt)
        np.random.seed(9)
        quiet(nf.noisefit, "config-data", "config-noise", stopat=2, olhcmult=10, samples=50)
        emuc.Posterior, np.linalg.cholesky, np.random.randn, np.savetxt = (
            orig_post, orig_chol, orig_randn, orig_savetxt)
        out = {"X": X, "y": y, "noise_inputs": np.loadtxt("noise-inputs"),
               "noise_outputs": np.loadtxt("noise-outputs"), "x_range": np.loadtxt("x_range_input"),
               "n_post": np.array(len(posts)), "n_draws": np.array(len(draws)),
               "n_chol": np.array(len(chols))}
        for i, z in enumerate(zps):
            out[f"zp{i}"] = z
        for i, p in enumerate(posts):
            for k, v in p.items():
                out[f"p{i}_{k}"] = v
        for i, L in enumerate(chols):
            out[f"chol{i}"] = L
        out["draws"] = np.concatenate([np.ravel(u) for u in draws])
        out["draw_sizes"] = np.array([np.size(u) for u in draws])
        for f in ("config-data", "config-noise", "beliefs-data", "beliefs-noise"):
            out["in_" + f.replace("-", "_")] = np.array(open(f).read())
        for f in ("beliefs-data-0f", "beliefs-noise-0f"):
            out[f.replace("-", "_")] = np.array(open(f).read())
        save("noise_fit.npz", **out)
    finally:
        emuc.Posterior, np.linalg.cholesky, np.random.randn, np.savetxt = (
            orig_post, orig_chol, orig_randn, orig_savetxt)
        os.chdir(cwd)
        shutil.rmtree(tmp)


if __name__ == "__main__":
    which = sys.argv[1:] or ["G1", "G2", "G3", "G4", "G5", "G6", "G7", "G8", "G9"]
    for w in which:
        print("==", w)
        {"G1": make_g1, "G2": make_g2, "G3": make_g3, "G4": make_g4, "G5": make_g5,
         "G6": make_g6, "G7": make_g7, "G8": make_g8, "G9": make_g9}[w]()
