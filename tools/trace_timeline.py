"""Timeline summary of one objective evaluation from a rocprofv3 kernel trace (dev tool).

usage: python3 tools/trace_timeline.py TRACE.csv [EVAL_INDEX]
Evaluations are split at the covariance-build kernel (k_dist_kbuild / k_pairs).  Per
evaluation: wall span, time with no kernel running, time with exactly one kernel running
(the chain alone), and per stream the busy time and launch count.
"""
import csv
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    which = int(sys.argv[2]) if len(sys.argv) > 2 else -1
    rows.sort(key=lambda r: int(r['Start_Timestamp']))
    starts = [i for i, r in enumerate(rows) if 'kbuild' in r['Kernel_Name'] or 'k_pairs' in r['Kernel_Name']]
    i0 = starts[which]
    i1 = starts[which + 1] if which != -1 and which + 1 < len(starts) else len(rows)
    ev = rows[i0:i1]
    iv = [(int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Queue_Id'], r['Kernel_Name']) for r in ev]
    t0 = min(a for a, _, _, _ in iv)
    t1 = max(b for _, b, _, _ in iv)
    pts = sorted([(a, 1) for a, _, _, _ in iv] + [(b, -1) for _, b, _, _ in iv])
    depth, last, idle, single = 0, t0, 0, 0
    for t, d in pts:
        if depth == 0:
            idle += t - last
        elif depth == 1:
            single += t - last
        depth += d
        last = t
    print(f"span {(t1 - t0) / 1e6:.2f} ms, idle {idle / 1e6:.2f} ms, one kernel only {single / 1e6:.2f} ms, "
          f"{len(iv)} launches")
    by = {}
    for a, b, q, n in iv:
        s = by.setdefault(q, [0, 0, {}])
        s[0] += b - a
        s[1] += 1
        k = n.split('(')[0][-48:]
        s[2][k] = s[2].get(k, 0) + (b - a)
    for q, (busy, cnt, names) in sorted(by.items()):
        top = sorted(names.items(), key=lambda x: -x[1])[:4]
        print(f"  queue {q}: busy {busy / 1e6:.2f} ms, {cnt} launches; " +
              ", ".join(f"{k} {v / 1e6:.2f}" for k, v in top))


if __name__ == '__main__':
    main()
