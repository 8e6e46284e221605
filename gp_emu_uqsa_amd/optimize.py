"""Hyperparameter optimisation (reference: _emulatoroptimise.py, class Optimize).

scipy's L-BFGS-B stays the host driver, exactly as in the reference
(:227-278, jac=True, same bounds and constraint sets); the objective it calls is
one synchronous gpe_objective per evaluation.  NotPositiveDefinite is mapped to
the reference's ``return None`` (:374-376, :489-491), which makes scipy raise
TypeError and the multistart loop move on to the next guess (:248-251).

Multistart tries are independent units: in a job with world_size > 1 (the group
of rendezvous.init_from_env(), or a torch.distributed group the caller set up)
the tries are sharded over ranks (one GPU per rank, no data exchange) and only
the (fun, x) results are gathered (replicas.py) -- the guess grid is drawn
identically on every rank, so the chosen optimum equals the sequential one.
With distributed.enable_objective() each evaluation is instead spread over all
ranks (row-block partition) and every rank runs every try in lockstep.
On one GPU, large problems run two tries at a time on two contexts
(Optimize._concurrency): the evaluations' idle CUs overlap.
"""
from __future__ import annotations

import os
import threading

import numpy as np
from scipy.optimize import minimize

from . import distributed
from . import native
from .model import upload_training
from . import replicas


class Optimize:
    def __init__(self, data, basis, par, beliefs, config):
        self.data = data
        self.basis = basis
        self.par = par
        self.beliefs = beliefs
        self.config = config
        self.print_message = False
        print("\n*** Optimization options ***")
        ndim = self.data.inputs.shape[1]
        d_b, n_b, s_b = [], [], []
        if config.delta_bounds == []:
            print("Data-based bounds for delta:")
            for i in range(ndim):
                rng = np.amax(self.data.inputs[:, i]) - np.amin(self.data.inputs[:, i])
                d_b.append([0.001, rng])
                print("    delta", i, "[{:04.4f} , {:04.4f}]".format(d_b[i][0], d_b[i][1]))
        else:
            print("User provided bounds for delta:")
            if len(config.delta_bounds) != ndim:
                print("ERROR: Wrong number of delta_bounds specified, exiting.")
                raise SystemExit(1)
            for i in range(ndim):
                if config.delta_bounds[i] == []:
                    rng = np.amax(self.data.inputs[:, i]) - np.amin(self.data.inputs[:, i])
                    d_b.append([0.001, rng])
                    tag = "(data)"
                else:
                    d_b.append(config.delta_bounds[i])
                    tag = "(user)"
                print("    delta", i, "[{:04.4f} , {:04.4f}]".format(d_b[i][0], d_b[i][1]), tag)
        if config.nugget_bounds == []:
            print("Data-based bounds for nugget:")
            n_b.append([0.0001, 0.01])
        else:
            print("User provided bounds for nugget:")
            n_b = config.nugget_bounds
        print("    nugget ", "[{:04.4f} , {:04.4f}]".format(n_b[0][0], n_b[0][1]))
        if config.sigma_bounds == []:
            print("Data-based bounds for sigma:")
            rng = np.sqrt(np.amax(self.data.outputs) - np.amin(self.data.outputs))
            s_b.append([0.001, rng])
        else:
            print("User provided bounds for sigma:")
            s_b = config.sigma_bounds
        print("    sigma  ", "[{:04.4f} , {:04.4f}]".format(s_b[0][0], s_b[0][1]))
        fit_nug = self.beliefs.fix_nugget == "F"
        mucm = self.beliefs.mucm == "T"
        config.bounds = tuple(d_b + (n_b if fit_nug else []) + ([] if mucm else s_b))
        if config.constraints == "bounds":
            self.bounds_constraint(config.bounds)
        else:
            self.standard_constraint(config.bounds)

    # -- constraint sets (reference :114-152)
    def _n_params(self):
        n = np.asarray(self.data.K.d).size
        if self.beliefs.fix_nugget == "F":
            n += 1
        if self.beliefs.mucm == "F":
            n += 1
        return n

    def standard_constraint(self, bounds):
        print("Setting up standard constraint")
        self.cons = [[self.data.K.transform(0.001), None] for _ in range(np.asarray(self.data.K.d).size)]
        if self.beliefs.fix_nugget == "F":
            self.cons.append([None, None])
        if self.beliefs.mucm == "F":
            self.cons.append([None, None])

    def bounds_constraint(self, bounds):
        print("Setting up bounds constraint")
        self.cons = [[self.data.K.transform(lo), self.data.K.transform(hi)]
                     for lo, hi in bounds[:self._n_params()]]

    # -- driver (reference :155-300)
    def llh_optimize(self, print_message=False):
        self.print_message = print_message
        print("Optimising hyperparameters...")
        bounds = self.data.K.transform(self.config.bounds)
        self.optimal(self.config.tries, bounds)
        print("best hyperparameters: ")
        self.data.K.print_kernel()
        print("sigma:", np.round(self.par.sigma, decimals=6))
        if self.beliefs.fix_nugget == "F":
            if self.beliefs.alt_nugget == "F":
                noisesig = np.sqrt(self.par.sigma ** 2 * self.par.nugget / (1.0 - self.par.nugget))
                print("'noise sigma' estimate from nugget:", noisesig)
            else:
                print("'noise sigma' estimate from alt nugget:", self.par.sigma * self.par.nugget)
        self.optimalbeta()
        print("best beta: ", self.par.beta)

    def _minimize(self, x_guess):
        fn = self.loglikelihood_mucm if self.beliefs.mucm == "T" else self.loglikelihood_gp4ml
        if self.config.constraints != "none":
            return minimize(fn, x_guess, method="L-BFGS-B", jac=True, bounds=self.cons)
        return minimize(fn, x_guess, method="L-BFGS-B", jac=True)

    def _run_try(self, x_guess):
        """One L-BFGS-B chain; None when it hit a non-PD matrix (the reference's
        TypeError -> "Trying next guess" path, :248-251)."""
        try:
            res = self._minimize(list(x_guess))
        except TypeError:
            return None
        return (float(res.fun), np.array(res.x, dtype=float), res)

    def _concurrency(self, ntries):
        """Chains in flight at once on this rank's GPU.  GPEMU_CONCURRENT_TRIES=k
        forces k (1: sequential); by default 2 when n >= 4096 and there are >= 2
        tries: one evaluation's latency-bound Cholesky steps leave CUs idle that a
        second chain's evaluation fills (+10% evaluations/s at n=16384).  Never
        with the row-block distributed objective (each evaluation is collective)."""
        if distributed.active_objective() is not None or ntries < 2:
            return 1
        env = os.environ.get("GPEMU_CONCURRENT_TRIES")
        if env is not None:
            return max(1, min(int(env), ntries))
        n = self.data.inputs.shape[0]
        return 2 if 4096 <= n <= 32768 else 1

    def _run_concurrent(self, items, guessgrid, k):
        """Tries dealt round-robin over k host threads, each bound to its own
        context (own HIP stream and workspaces) on the same GPU.  Every chain is
        the same deterministic computation as in the sequential loop, so results
        are identical; only the wall clock (and the order of "not PSD" messages)
        changes.  The objective's host-side bookkeeping (K.set_params, par.sigma)
        is overwritten from the best x after the loop, as in the sequential path."""
        ctxs = native.worker_contexts(k)
        r = None if np.isscalar(self.data.r) else self.data.r
        for c in ctxs:
            c.ensure_data(self.data.inputs, self.data.outputs, self.data.H, r)
        results, errors = {}, []

        def work(w):
            try:
                with native.bind_context(ctxs[w]):
                    for C in items[w::k]:
                        results[C] = self._run_try(guessgrid[:, C])
            except BaseException as e:   # re-raised on the caller's thread
                errors.append(e)

        threads = [threading.Thread(target=work, args=(w,)) for w in range(k)]
        for t in threads:
            t.start()
        for t in threads:
            t.join()
        if errors:
            raise errors[0]
        return results

    def optimal(self, numguesses, bounds):
        params = self._n_params()
        guessgrid = np.zeros([params, numguesses])
        print("Calculating initial guesses from bounds")
        for R in range(params):
            lo, hi = bounds[R][0], bounds[R][1]
            guessgrid[R, :] = lo + (hi - lo) * np.random.random_sample(numguesses)
        if self.beliefs.fix_nugget == "F":
            print("Training nugget on data")
        if self.beliefs.mucm == "T":
            print("Using MUCM method for sigma")
        if self.config.constraints != "none":
            print("Using L-BFGS-G method (with constraints)...")
        else:
            print("Using L-BFGS-G method (no constraints)...")

        if distributed.active_objective() is None:
            upload_training(self.data)
        items = replicas.my_items(numguesses)
        k = self._concurrency(len(items))
        if k > 1:
            results = self._run_concurrent(items, guessgrid, k)
        else:
            results = {}
            for C in items:
                results[C] = self._run_try(guessgrid[:, C])
        results = replicas.gather_results(results, numguesses)

        first_try, best_min, best_x = True, 10000000.0, None
        for C in range(numguesses):
            r = results.get(C)
            if r is None:
                print("Trying next guess...")
                continue
            fun, x, res = r
            if self.print_message and res is not None:
                print(res, "\n")
                if res.success is not True:
                    print(res.message, "Not succcessful.")
            sig_str = ""
            if self.beliefs.mucm == "T":
                self.sigma_analytic_mucm(self.data.K.untransform(x))
                sig_str = "  sig: " + str(np.around(self.par.sigma, decimals=4))
            print("  hp: ", np.around(self.data.K.untransform(x), decimals=4),
                  " llh: ", -1.0 * np.around(fun, decimals=4), sig_str)
            if fun < best_min or first_try:
                best_min = fun
                best_x = self.data.K.untransform(x)
                first_try = False
        print("********")
        if first_try:
            print("ERROR: No optimization was made due to non-PSD errors. Increase 'tries'. Exiting.")
            raise SystemExit(1)
        if self.beliefs.mucm == "T":
            self.data.K.set_params(best_x)
            self.par.delta = self.data.K.d
            self.par.nugget = self.data.K.n
            self.sigma_analytic_mucm(best_x)
        else:
            self.data.K.set_params(best_x[:-1])
            self.par.delta = self.data.K.d
            self.par.nugget = self.data.K.n
            self.par.sigma = best_x[-1]
        s2 = self.par.sigma ** 2
        self.data.make_A(s2)
        self.data.make_H()

    # -- objectives: one gpe_objective call each
    def _call(self, variant, x, want_grad=True):
        obj = distributed.active_objective()
        if obj is not None:   # collective row-block objective (distributed.enable_objective)
            r = None if np.isscalar(self.data.r) else self.data.r
            obj.ensure_data(self.data.inputs, self.data.outputs, self.data.H, r)
            ctx = obj
        else:
            ctx = native.default_context()
        return ctx.objective(variant, self.data.K.kind, x, nu_fixed=float(self.data.K.n),
                             want_grad=want_grad)

    def loglikelihood_mucm(self, x):
        """MUCM -LLH and gradient (reference :305-378; gradient carries the
        reference's sigma-hat^2 factor)."""
        x = self.data.K.untransform(x)
        self.data.K.set_params(x)
        self.data.make_A()
        try:
            llh, grad, sig2 = self._call(native.MUCM, x)
        except native.NotPositiveDefinite:
            print("  Matrix not PSD for", x, ", try adjusting nugget.")
            return None
        self.par.sigma = np.sqrt(sig2)
        return llh, grad

    def sigma_analytic_mucm(self, x):
        """sigma-hat from the analytic MUCM estimate (reference :382-408)."""
        self.data.K.set_params(x)
        self.data.make_A()
        try:
            _, _, sig2 = self._call(native.MUCM, np.asarray(x, dtype=float), want_grad=False)
        except native.NotPositiveDefinite:
            print("  In sigma_analytic_mucm(): Matrix not PSD for", x, ", try adjusting nugget.")
            raise SystemExit(1)
        self.par.sigma = np.sqrt(sig2)

    def loglikelihood_gp4ml(self, x):
        """gp4ml -LLH and gradient (reference :412-493)."""
        x = self.data.K.untransform(x)
        self.data.K.set_params(x[:-1])
        self.par.sigma = x[-1]
        self.data.make_A(x[-1] ** 2)
        try:
            llh, grad, _ = self._call(native.GP4ML, x)
        except native.NotPositiveDefinite:
            print("  Matrix not PSD for", x, ", try adjusting nugget.")
            return None
        return llh, grad

    def optimalbeta(self):
        """GLS beta with the current A (reference :497-504)."""
        ctx = upload_training(self.data)
        ctx.ensure_factor(self.data.K.kind, self.data.K.d, float(self.data.K.n), 1.0,
                          self.data.r_scale())
        self.par.beta = ctx.beta()
