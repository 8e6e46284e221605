"""History matching with batched posteriors.

Mirrors gp_emu_uqsa.history_match (history_match/history_match.py,
_hmutilfunctions.py): imp_plot, imp_plot_recon, nonimp_data and new_wave_design keep
the reference's arguments, printed progress, RNG use (one optLatinHyperCube per input
pair or wave) and files (`<m>_IMP_<i>_<j>`, `<m>_ODP_<i>_<j>`, `nonimp_`/`noninp_`,
the wave design).

The difference is how posteriors are called:
- imp_plot: the reference builds one Posterior per grid cell and emulator
  (history_match.py:91-121) and forms each cell's full n x n variance for its diagonal.
  Here every cell of an input pair goes into ONE diagonal-variance posterior per emulator
  (grid^2 * n points), streamed through gpe_posterior.
- nonimp_data / new_wave_design: one posterior per emulator, diagonal only.

Implausibility I = |mean - z| / sqrt(var + var_extra). Per point, the maxno largest over
emulators are taken. Per cell, IMP is their minimum over points and ODP the fraction
below cm (:123-136).

Plots use today's matplotlib: `set_facecolor` and `adjustable='box'` replace the removed
`set_axis_bgcolor` and `'box-forced'` of _hmutilfunctions.py:81,102.
"""
from __future__ import annotations

import numpy as _np

from . import design_inputs as _gd
from . import model as _model


# ----------------------------------------------------------------- helpers (_hmutilfunctions.py)
def make_sets(ai):
    sets = []
    for i in ai:
        for j in ai:
            if i != j and i < j and [i, j] not in sets:
                sets.append([i, j])
    return sets


def emulsetup(emuls):
    minmax, orig_minmax = {}, {}
    sets = []
    for e in emuls:
        try:
            ai = e.beliefs.active_index
            mm = e.beliefs.input_minmax
        except AttributeError:
            print("ERROR: Emulator(s) were not previously trained and reconstructed "
                  "using updated beliefs files, "
                  "so they are missing 'active_index' and 'input_minmax'. Exiting.")
            raise SystemExit
        sets = make_sets(ai)
        for i in range(len(ai)):
            minmax[str(ai[i])] = list((_np.array(mm[i]) - mm[i][0]) / (mm[i][1] - mm[i][0]))
            orig_minmax[str(ai[i])] = list(_np.array(mm[i]))
    print("\nactive index pairs:", sets)
    print("\nminmax for active inputs:", minmax)
    print("original units minmax for active inputs:", orig_minmax)
    return sets, minmax, orig_minmax


def ref_act(minmax):
    act_ref = {key: c for c, key in enumerate(sorted(minmax.keys(), key=lambda x: int(x)))}
    print("\nrelate active_indices to integers:", act_ref)
    return act_ref


def ref_plt(act):
    plt_ref = {str(key): c for c, key in enumerate(sorted(act))}
    print("\nrelate restricted active_indices to subplot indices:", plt_ref)
    return plt_ref


def check_act(act, sets):
    if type(act) is not list:
        print("ERROR: 'act' argument must be a list, but", act, "was supplied. Exiting.")
        raise SystemExit
    flat = [item for sublist in sets for item in sublist]
    for a in act:
        if a not in flat:
            print("ERROR: index", a, "in 'act' is not an active_index of the emulator(s). Exiting.")
            raise SystemExit
    return True


def load_datafiles(datafiles, orig_minmax):
    try:
        sim_x, sim_y = _np.loadtxt(datafiles[0]), _np.loadtxt(datafiles[1])
    except FileNotFoundError:
        print("ERROR: datafile(s)", datafiles, "for inputs and/or outputs not found. Exiting.")
        raise SystemExit
    for key in orig_minmax.keys():
        sim_x[:, int(key)] = (sim_x[:, int(key)] - orig_minmax[key][0]) \
            / (orig_minmax[key][1] - orig_minmax[key][0])
    return sim_x, sim_y


def _posterior_diag(E, x_active):
    """Posterior mean and variance diagonal of emulator E at points x (its active
    inputs, scaled), one batched GPU call (reference: Data + Posterior per call site)."""
    ni = _model.Data(x_active, None, E.basis, E.par, E.beliefs, E.K)
    post = _model.Posterior(ni, E.training, E.par, E.beliefs, E.K, predict=True, full_var=False)
    return post.mean, post.var


def _imaxes(I2, maxno):
    """Per point, the maxno largest implausibilities over emulators, ascending."""
    I = _np.sqrt(I2)
    return _np.sort(_np.partition(I, -maxno, axis=1)[:, -maxno:], axis=1)


# ----------------------------------------------------------------- plotting
def make_plots(s, plt_ref, cm, maxno, ax, IMP, ODP, minmax=None, recon=False):
    import matplotlib.pyplot as _plt
    imp_pal = _plt.get_cmap('jet')
    odp_pal = _plt.get_cmap('afmhot')
    (odp, imp) = (ODP, IMP) if recon else (ODP[maxno - 1], IMP[maxno - 1])
    ax[plt_ref[str(s[0])], plt_ref[str(s[1])]].set_facecolor('darkgray')
    ex = None if recon else (minmax[str(s[0])][0], minmax[str(s[0])][1],
                             minmax[str(s[1])][0], minmax[str(s[1])][1])
    im_imp = ax[plt_ref[str(s[1])], plt_ref[str(s[0])]].imshow(
        imp.T, origin='lower', cmap=imp_pal, extent=ex, vmin=0.0, vmax=cm + 1, interpolation='none')
    im_odp = ax[plt_ref[str(s[0])], plt_ref[str(s[1])]].imshow(
        _np.ma.masked_where(odp == 0, odp).T, origin='lower', cmap=odp_pal, extent=ex, vmin=0.0,
        vmax=1.0, interpolation='none')
    _plt.colorbar(im_imp, ax=ax[plt_ref[str(s[1])], plt_ref[str(s[0])]])
    _plt.colorbar(im_odp, ax=ax[plt_ref[str(s[0])], plt_ref[str(s[1])]])


def plot_options(plt_ref, ax, fig, minmax=None):
    import matplotlib.pyplot as _plt
    for key in plt_ref:
        ax[plt_ref[key], plt_ref[key]].set(adjustable='box', aspect='equal')
        if minmax is not None:
            ax[plt_ref[key], plt_ref[key]].text(.25, .5, "Input " + str(key) + "\n"
                                                + str(minmax[key][0]) + "\n-\n" + str(minmax[key][1]))
        fig.delaxes(ax[plt_ref[key], plt_ref[key]])
    for a in ax.flat:
        a.set_xticks([])
        a.set_yticks([])
        a.set_aspect('equal')
    _plt.tight_layout()


# ----------------------------------------------------------------- API (history_match.py)
def imp_plot(emuls, zs, cm, var_extra, maxno=1, olhcmult=100, grid=10, act=[], fileStr="", plot=True):
    """Implausibility (lower triangle) and optical depth (upper triangle) per pair of
    active inputs over a grid x grid mesh, each cell sampled by an oLHC design of the
    other inputs (reference :7-150).  Writes <m>_IMP_<i>_<j> / <m>_ODP_<i>_<j>."""
    sets, minmax, orig_minmax = emulsetup(emuls)
    check_act(act, sets)
    act_ref = ref_act(minmax)
    plt_ref = ref_plt(act)
    num_inputs = len(minmax)
    dim = num_inputs - 2
    maxno = int(maxno)
    IMP = [_np.zeros((grid, grid)) for _ in range(maxno)]
    ODP = [_np.zeros((grid, grid)) for _ in range(maxno)]
    print("Creating plot objects... may take some time...")
    plot = plot is True
    rc = num_inputs if act == [] else len(act)
    fig = ax = None
    if plot:
        import matplotlib.pyplot as _plt
        fig, ax = _plt.subplots(nrows=rc, ncols=rc)
    plt_ref = act_ref if act == [] else ref_plt(act)
    less_sets = sets if act == [] else [s for s in sets if s[0] in act and s[1] in act]
    print("HM for input pairs:", less_sets)

    for s in less_sets:
        print("\nset:", s)
        X1 = _np.linspace(minmax[str(s[0])][0], minmax[str(s[0])][1], grid, endpoint=False)
        X1 = X1 + 0.5 * (minmax[str(s[0])][1] - minmax[str(s[0])][0]) / float(grid)
        X2 = _np.linspace(minmax[str(s[1])][0], minmax[str(s[1])][1], grid, endpoint=False)
        X2 = X2 + 0.5 * (minmax[str(s[1])][1] - minmax[str(s[1])][0]) / float(grid)
        print("Values of the grid 1:", X1)
        print("Values of the grid 2:", X2)
        n = dim * int(olhcmult)
        N = int(n / 2)
        olhc_range = [it[1] for it in sorted(minmax.items(), key=lambda x: int(x[0]))
                      if int(it[0]) != s[0] and int(it[0]) != s[1]]
        print("olhc_range:", olhc_range)
        filename = "imp_input_" + str(s[0]) + '_' + str(s[1])
        _gd.optLatinHyperCube(dim, n, N, olhc_range, filename)
        x_other = _np.loadtxt(filename)
        # every grid cell at once: cell c = i*grid + j owns rows [c n, (c+1) n)
        cells = grid * grid
        x = _np.empty((cells * n, num_inputs))
        c0 = _np.repeat(_np.repeat(X1, grid), n)
        c1 = _np.repeat(_np.tile(X2, grid), n)
        x[:, act_ref[str(s[0])]] = c0
        x[:, act_ref[str(s[1])]] = c1
        other_dim = [act_ref[str(key)] for key in act_ref if int(key) not in s]
        xo = x_other.reshape(n, -1) if x_other.ndim > 1 else x_other.reshape(n, 1)
        x[:, other_dim] = _np.tile(xo, (cells, 1))
        print("\nCalculating Implausibilities...")
        I2 = _np.zeros((cells * n, len(emuls)))
        for o in range(len(emuls)):
            E, z, var_e = emuls[o], zs[o], var_extra[o]
            Eai = E.beliefs.active_index
            if s[0] in Eai and s[1] in Eai:
                act_ind_list = [act_ref[str(l)] for l in Eai]
                mean, var = _posterior_diag(E, x[:, act_ind_list])
                I2[:, o] = (mean - z) ** 2 / (var + var_e)
        Imaxes = _imaxes(I2, maxno).reshape(cells, n, maxno)
        for m in range(maxno):
            col = Imaxes[:, :, -(m + 1)]
            IMP[m][:, :] = col.min(axis=1).reshape(grid, grid)
            ODP[m][:, :] = (col < cm).sum(axis=1).reshape(grid, grid) / float(n)
        nfileStr = fileStr + "_" if fileStr != "" else fileStr
        for m in range(maxno):
            _np.savetxt(nfileStr + str(m + 1) + "_" + "IMP_" + str(s[0]) + '_' + str(s[1]), IMP[m])
            _np.savetxt(nfileStr + str(m + 1) + "_" + "ODP_" + str(s[0]) + '_' + str(s[1]), ODP[m])
        if plot:
            make_plots(s, plt_ref, cm, maxno, ax, IMP, ODP, minmax=minmax)
    if plot:
        import matplotlib.pyplot as _plt
        plot_options(plt_ref, ax, fig, minmax)
        _plt.show()
    return


def imp_plot_recon(cm, maxno=1, act=[], fileStr=""):
    """Re-plot from the files imp_plot wrote (reference :153-192)."""
    if act == []:
        print("WARNING: Please specificy 'act' for active inputs. Return None.")
        return None
    import matplotlib.pyplot as _plt
    print("Creating plot objects... may take some time...")
    fig, ax = _plt.subplots(nrows=len(act), ncols=len(act))
    plt_ref = ref_plt(act)
    sets = make_sets(act)
    print("HM for input pairs:", sets)
    for s in sets:
        print("\nset:", s)
        nfileStr = fileStr + "_" if fileStr != "" else fileStr
        IMP = _np.loadtxt(nfileStr + str(maxno) + "_" + "IMP_" + str(s[0]) + '_' + str(s[1]))
        ODP = _np.loadtxt(nfileStr + str(maxno) + "_" + "ODP_" + str(s[0]) + '_' + str(s[1]))
        make_plots(s, plt_ref, cm, maxno, ax, IMP, ODP, recon=True)
    plot_options(plt_ref, ax, fig)
    _plt.show()
    return


def _implausible_rows(emuls, zs, var_extra, x, act_ref, maxno, cm):
    I2 = _np.zeros((x.shape[0], len(emuls)))
    for o in range(len(emuls)):
        E, z, var_e = emuls[o], zs[o], var_extra[o]
        act_ind_list = [act_ref[str(l)] for l in E.beliefs.active_index]
        mean, var = _posterior_diag(E, x[:, act_ind_list])
        I2[:, o] = (mean - z) ** 2 / (var + var_e)
    Imaxes = _imaxes(I2, maxno)
    return Imaxes[:, -maxno] < cm


def nonimp_data(emuls, zs, cm, var_extra, datafiles, maxno=1, act=[], fileStr=""):
    """Keep the non-implausible rows of a data set (reference :195-256).  Writes
    `nonimp_<inputs file>` (scaled inputs, as the reference) and `noninp_<outputs file>`."""
    sets, minmax, orig_minmax = emulsetup(emuls)
    act_ref = ref_act(minmax)
    check_act(act, sets)
    maxno = int(maxno)
    sim_x, sim_y = load_datafiles(datafiles, orig_minmax)
    print("\nCalculating Implausibilities...")
    keep = _implausible_rows(emuls, zs, var_extra, sim_x, act_ref, maxno, cm)
    nimp_inputs, nimp_outputs = sim_x[keep], sim_y[keep]
    nfileStr = fileStr + "_" if fileStr != "" else fileStr
    _np.savetxt(nfileStr + "nonimp_" + datafiles[0], nimp_inputs)
    _np.savetxt(nfileStr + "noninp_" + datafiles[1], nimp_outputs)
    print(len(nimp_inputs), "data points were non-implausible")
    return len(nimp_inputs)


def new_wave_design(emuls, zs, cm, var_extra, datafiles, maxno=1, olhcmult=100, act=[], fileStr=""):
    """Non-implausible points of a new oLHC design optimised against the given
    (non-implausible) data (reference :259-339).  Writes `<fileStr_><inputs file>`."""
    sets, minmax, orig_minmax = emulsetup(emuls)
    act_ref = ref_act(minmax)
    check_act(act, sets)
    dim = len(minmax)
    maxno = int(maxno)
    sim_x, sim_y = load_datafiles(datafiles, orig_minmax)
    n = dim * int(olhcmult)
    N = int(n / 2)
    olhc_range = [it[1] for it in sorted(minmax.items(), key=lambda x: int(x[0]))]
    print("olhc_range:", olhc_range)
    filename = "olhc_des"
    _gd.optLatinHyperCube(dim, n, N, olhc_range, filename, fextra=sim_x)
    x = _np.loadtxt(filename)
    if x.ndim == 1:
        x = x.reshape(-1, 1)
    print("\nCalculating Implausibilities...")
    keep = _implausible_rows(emuls, zs, var_extra, x, act_ref, maxno, cm)
    nimp_inputs = x[keep]
    nfileStr = fileStr + "_" if fileStr != "" else fileStr
    _np.savetxt(nfileStr + datafiles[0], nimp_inputs)
    print("Generated", len(nimp_inputs), "new data points")
    return len(nimp_inputs)
