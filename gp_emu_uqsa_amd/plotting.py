"""Posterior plots (reference: emulatorfunctions.plot :128-223 and
_emulatorplotting.py).  Visualisation only: the grid's posterior comes from the
GPU path with the diagonal-only variance (the reference forms the full 900 x 900
covariance and then takes its diagonal, _emulatorplotting.py:51)."""
from __future__ import annotations

import numpy as np

from . import model as _model

GRID = 30   # points per plotted dimension (reference: pn=30)


def make_inputs(dim, rows, cols, plot_dims, fixed_dims, fixed_vals, one_d, minmax):
    """Prediction grid (reference _emulatorplotting.make_inputs)."""
    if dim >= 2 and not one_d:
        X1 = np.linspace(minmax[0][0], minmax[0][1], rows)
        X2 = np.linspace(minmax[1][0], minmax[1][1], cols)
        x_all = np.zeros((rows * cols, dim))
        x_all[:, plot_dims[0]] = np.repeat(X1, cols)
        x_all[:, plot_dims[1]] = np.tile(X2, rows)
        if dim > 2:
            for i in range(len(fixed_dims)):
                x_all[:, fixed_dims[i]] = fixed_vals[i]
    elif dim >= 2:
        x_all = np.zeros((rows * cols, dim))
        x_all[:, plot_dims[0]] = np.linspace(minmax[0][0], minmax[0][1], rows * cols)
        for i in range(len(fixed_dims)):
            x_all[:, fixed_dims[i]] = fixed_vals[i]
    else:
        x_all = np.linspace(minmax[0][0], minmax[0][1], rows * cols).reshape(-1, 1)
    return x_all


def _labels(E, plot_dims, customLabels, one_d, dim):
    default_x = "input " + str(plot_dims[0])
    if one_d:
        default_y = "output " + str(E.beliefs.output)
    else:
        default_y = "output " if dim == 1 else "input " + str(plot_dims[1])
    xl = customLabels[0] if len(customLabels) > 0 else default_x
    yl = customLabels[1] if len(customLabels) > 1 else default_y
    return xl, yl


def plot(E, plot_dims, fixed_dims=[], fixed_vals=[], mean_or_var="mean", customLabels=[],
         points=False, predict=True):
    import matplotlib.pyplot as plt

    dim = E.training.inputs[0].size
    print("\n*** Generating plot ***")
    one_d = len(plot_dims) == 1 and dim > 1
    x, y = [], []
    if points and mean_or_var == "mean":
        x = E.training.inputs[:, plot_dims[0]]
        y = E.training.outputs
    minmax = [[np.amin(E.training.inputs[:, plot_dims[0]]), np.amax(E.training.inputs[:, plot_dims[0]])]]
    if not one_d and dim > 1:
        minmax.append([np.amin(E.training.inputs[:, plot_dims[1]]),
                       np.amax(E.training.inputs[:, plot_dims[1]])])
    xlabel, ylabel = _labels(E, plot_dims, customLabels, one_d, dim)
    grid = make_inputs(dim, GRID, GRID, plot_dims, fixed_dims, fixed_vals, one_d, minmax)
    newinputs = _model.Data(grid, None, E.basis, E.par, E.beliefs, E.K)
    print("Prediction (rather than estimation)" if predict else "Estimation (rather than prediction)")
    post = _model.Posterior(newinputs, E.training, E.par, E.beliefs, E.K, predict, full_var=False)
    pred = post.mean if mean_or_var != "var" else post.var
    if dim >= 2 and not one_d:
        Z = pred.reshape(GRID, GRID)
        print("Plotting... output range:", np.around(np.amin(Z), decimals=4), "to",
              np.around(np.amax(Z), decimals=4))
        plt.figure()
        plt.xlabel(xlabel)
        plt.ylabel(ylabel)
        ax = plt.gca()
        im = ax.imshow(Z.T, origin="lower", cmap=plt.get_cmap("rainbow"),
                       extent=(minmax[0][0], minmax[0][1], minmax[1][0], minmax[1][1]))
        ext = im.get_extent()
        ax.set_aspect(abs((ext[1] - ext[0]) / (ext[3] - ext[2])))
        plt.colorbar(im)
        plt.show()
    else:
        print("Plotting... output range:", np.around(np.amin(pred), decimals=4), "to",
              np.around(np.amax(pred), decimals=4))
        plt.plot(np.linspace(minmax[0][0], minmax[0][1], GRID * GRID), pred, linewidth=2.0)
        if len(x) and len(y):
            plt.plot(x, y, "x")
        plt.xlabel(xlabel)
        plt.ylabel(ylabel)
        plt.show()
    return post
