"""Kernel timeline of the last objective evaluation at one n (dev tool).

  rocprofv3 --kernel-trace --output-format csv -d DIR -o ev -- python3 tools/eval_timeline.py run N [reps]
  python3 tools/eval_timeline.py show DIR/.../ev_kernel_trace.csv reps

`run`: reps LLH + gradient evaluations at n = N, d = 10.  `show`: each kernel of the last
evaluation with its start (us after the evaluation's first kernel), duration and grid."""
import csv
import sys


def run(n, reps):
    import numpy as np
    sys.path.insert(0, ".")
    from gp_emu_uqsa_amd import native, synthetic
    ctx = native.Context(0)
    X, f, H = synthetic.problem(n, 10, seed=0)
    ctx.set_data(X, f, H)
    hp = np.concatenate([np.ones(10), [1e-3, 1.0]])
    for _ in range(reps):
        ctx.objective(0, 0, hp)
    ctx.close()


def show(path, reps):
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r['Start_Timestamp']))
    rows = rows[len(rows) - len(rows) // reps:]
    t0 = int(rows[0]['Start_Timestamp'])
    prev = t0
    for r in rows:
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        g = int(r['Grid_Size_X']) // max(1, int(r['Workgroup_Size_X']))
        print('%8.1f  +%6.1f  %7.1f us  grid %6d  %s' % ((s - t0) / 1e3, (s - prev) / 1e3, (e - s) / 1e3, g,
                                                       r['Kernel_Name'].split('(')[0][-48:]))
        prev = e
    print('evaluation: %.1f us' % ((int(rows[-1]['End_Timestamp']) - t0) / 1e3))


if __name__ == "__main__":
    if sys.argv[1] == "run":
        run(int(sys.argv[2]), int(sys.argv[3]) if len(sys.argv) > 3 else 5)
    else:
        show(sys.argv[2], int(sys.argv[3]))
