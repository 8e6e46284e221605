"""Per-tile timeline of the fused Cholesky sweep (dev tool; the -DGEMM_TTRACE build):
  bash tools/tile_timeline.sh      (builds gp_emu_uqsa_amd/libgpemu_ttrace.so here)
  GPEMU_LIB=gp_emu_uqsa_amd/libgpemu_ttrace.so GPEMU_CHOL_PRIO=0 python tools/tile_timeline.py [stop]
The objective stops after Cholesky launch `stop` (GPEMU_DEBUG_STOP_STEP, default the last);
every workgroup of the sweep is traced in start order (start / end on the 100 MHz wall
clock, kind, K).  Per phase: the 512 workgroup slots' occupancy, the launches' spans and
the gaps between them, the drains (time a launch spends below 90% occupancy at its end)
and the tile durations.  -> gpurun_out/tile_timeline.json"""
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from gp_emu_uqsa_amd import native, synthetic  # noqa: E402

n = 16384
NB = n // 128
stop = int(sys.argv[1]) if len(sys.argv) > 1 else NB - 1   # < 0: the whole evaluation
tag = sys.argv[2] if len(sys.argv) > 2 else ""
ctx = native.Context(0)
X, f, H = synthetic.problem(n, 10, seed=0)
ctx.set_data(X, f, H)
hp = np.concatenate([np.ones(10), [1e-3, 1.0]])
ctx.objective(0, 0, hp)
ctx.objective(0, 0, hp)
lib = native.load_library()
lib.gpe_debug_ttrace.argtypes = [ctypes.c_void_p, ctypes.c_int32]
lib.gpe_debug_ttrace_count.argtypes = [ctypes.c_int32]
assert lib.gpe_debug_ttrace_count(1) >= 0
if stop >= 0:
    os.environ["GPEMU_DEBUG_STOP_STEP"] = str(stop)
    try:
        ctx.objective(0, 0, hp)
    except Exception:   # the debug stop
        pass
    os.environ.pop("GPEMU_DEBUG_STOP_STEP", None)
else:   # stop < 0: one whole evaluation; per launch after the Cholesky (TRTRI, LAUUM)
    ctx.objective(0, 0, hp)
cnt = lib.gpe_debug_ttrace_count(0)
assert 0 < cnt <= 262144, cnt
buf = np.zeros(8 * cnt, dtype=np.uint64)
assert lib.gpe_debug_ttrace(buf.ctypes.data, buf.size) == 0
w = buf.reshape(cnt, 8)
np.save(os.path.join(ROOT, "gpurun_out", f"tile_timeline{tag}.npy"), w)   # raw, for offline analysis
t0 = w[:, 0].min()
st = (w[:, 0] - t0) / 100.0
en = (w[:, 3].astype(np.float64) - t0) / 100.0
kind = (w[:, 6] & 3).astype(int)
bidx = (w[:, 6] >> 2).astype(int)
# launches: each starts with its workgroup 0, a diagonal tile (10 us of slack for the
# dispatch skew between XCDs); steps: the diagonal tiles in start order
starts0 = np.sort(st[(bidx == 0) & (kind == 1)]) - 10.0
launch = np.searchsorted(starts0, st, side="right") - 1
NL = len(starts0)
beg = np.array([st[launch == L].min() for L in range(NL)])
end = np.array([np.nanmax(en[launch == L]) for L in range(NL)])
dstart = np.sort(st[kind == 1])
total = float(np.nanmax(end))
grid = np.arange(0.0, total, 0.5)
ok = np.isfinite(en)
ev = np.concatenate([np.stack([st[ok], np.ones(ok.sum())], 1), np.stack([en[ok], -np.ones(ok.sum())], 1)])
ev = ev[np.argsort(ev[:, 0], kind="stable")]
cum = np.cumsum(ev[:, 1])
idx = np.searchsorted(ev[:, 0], grid, side="right") - 1
act = np.where(idx >= 0, cum[np.maximum(idx, 0)], 0)
drain = np.zeros(NL)
for L in range(NL):
    mm = (grid >= beg[L]) & (grid < end[L])
    full = np.nonzero(act[mm] >= 0.9 * 512)[0]
    drain[L] = (end[L] - grid[mm][full[-1]]) if len(full) else end[L] - beg[L]
out = {"stop": stop, "tiles": int(cnt), "launches": int(NL), "sweep_ms": total / 1e3,
       "occupancy": float(act.mean() / 512), "phases": {}}
bounds = [0.0] + [float(dstart[k]) for k in (48, 88) if k < len(dstart)] + [total]
names = ["steps 0-47", "steps 48-87", "steps 88-127"]
for i in range(len(bounds) - 1):
    a, b = bounds[i], bounds[i + 1]
    m = (grid >= a) & (grid < b)
    Ls = [L for L in range(NL) if a <= beg[L] < b]
    ph = {"ms": (b - a) / 1e3, "occupancy": float(act[m].mean() / 512), "launches": len(Ls),
          "drain_ms": float(drain[Ls].sum() / 1e3) if Ls else 0.0}
    for k, kn in ((0, "bulk"), (1, "diag"), (2, "panel")):
        sel = (kind == k) & (st >= a) & (st < b) & ok
        if sel.any():
            ph[kn + "_us"] = float(np.mean(en[sel] - st[sel]))
    out["phases"][names[i]] = ph
if stop < 0:   # the launches after the sweep: every launch starts with its workgroup 0
    s0 = np.sort(st[bidx == 0])
    after = s0[s0 > dstart[-1] + 1.0]
    rows = []
    for i, a in enumerate(after):
        b = after[i + 1] if i + 1 < len(after) else np.inf
        sel = (st >= a - 10.0) & (st < b - 10.0) & ok
        if not sel.any():
            continue
        lb, le = st[sel].min(), en[sel].max()
        mm = (grid >= lb) & (grid < le)
        full = np.nonzero(act[mm] >= 0.9 * 512)[0]
        rows.append({"tiles": int(sel.sum()), "span_us": float(le - lb),
                     "occupancy": float(act[mm].mean() / 512) if mm.any() else 0.0,
                     "drain_us": float(le - grid[mm][full[-1]]) if len(full) else float(le - lb),
                     "tile_us_mean": float(np.mean(en[sel] - st[sel])), "tile_us_max": float(np.max(en[sel] - st[sel])),
                     "K_max": int(w[sel, 7].max())})
    out["after_sweep"] = rows
print(json.dumps(out, indent=1))
json.dump(out, open(os.path.join(ROOT, "gpurun_out", f"tile_timeline{tag}.json"), "w"), indent=1)
