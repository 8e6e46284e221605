"""Predicted strong-scaling curve of the row-block objective (dev tool).

  python tools/dist_model.py --p1-ms MS --p1-value-ms MS [--points 16384] [--basis 11]

Counts, from the schedule of gpemu_dist.hip (column groups, recursive TRTRI chunks), the
collectives one LLH + gradient issues and the bytes each rank receives in them, then
predicts the evaluation time at P ranks over xGMI as

  T(P) = chain + sweep_bulk / P + (trtri + slab + rest) / P
         + sum over collectives of (alpha + received bytes / beta)

with the compute terms from the P = 1 loopback run (one GPU, no real collectives) and
alpha / beta the per-collective latency and per-rank receive bandwidth of RCCL over the
MI355X's xGMI (defaults: 25 us, 64 GB/s at P = 2 over one link, 300 GB/s at P >= 4).
The sweep's collectives sit on the chain (the look-ahead overlaps the bulk, not them)."""
import argparse
import json

TILE = 128
T2B = TILE * TILE * 8      # bytes per tile


def sweep_collectives(nb, na, P):
    """(count, bytes received per rank): Dinv broadcast + panel all-gather per step."""
    cnt, rb = 0, 0
    for k in range(nb):
        cnt += 1
        rb += T2B if P > 1 else 0                                  # Dinv from its owner
        tiles = nb + na - 1 - k                                     # panel tiles below k
        seg = -(-tiles // P)                                        # max per rank
        cnt += 1
        rb += (P - 1) * seg * T2B                                   # all-gather (padded segments)
    return cnt, rb


def trtri_collectives(nb, P, slab_rows):
    """(count, bytes received per rank) of the recursive TRTRI's chunked all-gathers."""
    n_pad = nb * TILE
    cap = slab_rows * TILE * n_pad * 8
    cnt, rb = 0, 0
    s = 2
    while s // 2 < nb:
        a = s // 2
        pairs = [(t0, t0 + a, min(t0 + s, nb)) for t0 in range(0, nb - a, s)]
        g1 = sum(a for _ in pairs)
        s1 = sum(-(-a // P) for _ in pairs)
        g2 = sum(t1 - h for (_, h, t1) in pairs)
        s2 = sum(-(-(t1 - h) // P) for (_, h, t1) in pairs)

        def fits(w):
            return g2 * w * T2B <= cap and (P == 1 or (g1 * w * T2B <= cap and P * s1 * w * T2B <= cap
                                                        and P * s2 * w * T2B <= cap))
        cc = a
        while cc > 1 and not fits(cc):
            cc = (cc + 1) // 2
        for j0 in range(0, a, cc):
            cw, rows1 = min(cc, a - j0), a - j0
            seg1 = sum(-(-rows1 // P) * cw for _ in pairs)
            seg2 = sum(cw * -(-(t1 - h) // P) for (_, h, t1) in pairs)
            if P > 1:
                cnt += 2
                rb += (P - 1) * (seg1 + seg2) * T2B
        s *= 2
    return cnt, rb


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=16384)
    ap.add_argument("--basis", type=int, default=11, help="q + 1")
    ap.add_argument("--p1-ms", type=float, default=None, help="loopback P=1 LLH+gradient ms")
    ap.add_argument("--p1-value-ms", type=float, default=None, help="loopback P=1 value-only ms")
    ap.add_argument("--chain-us", type=float, default=75.0, help="diagonal factor + panel per step, us")
    ap.add_argument("--alpha-us", type=float, default=25.0)
    ap.add_argument("--beta2", type=float, default=64.0, help="GB/s per rank at P=2")
    ap.add_argument("--beta", type=float, default=300.0, help="GB/s per rank at P>=4")
    args = ap.parse_args()
    nb = -(-args.points // TILE)
    na = -(-args.basis // TILE)
    n_pad = nb * TILE
    slab_rows = max(1, min(nb, (1 << 26) // (TILE * n_pad)))
    rows = []
    for P in (1, 2, 4, 8):
        c_sw, b_sw = sweep_collectives(nb, na, P)
        c_tr, b_tr = trtri_collectives(nb, P, slab_rows)
        c_rest = 6                                                  # Gram, logdet, info, Z, W, sums
        b_rest = (P - 1) / P * (n_pad * args.basis * 8 * 2) if P > 1 else 0
        beta = (args.beta2 if P == 2 else args.beta) * 1e9
        comm_sweep = 0.0 if P == 1 else c_sw * args.alpha_us * 1e-3 + b_sw / beta * 1e3
        comm_tr = 0.0 if P == 1 else c_tr * args.alpha_us * 1e-3 + b_tr / beta * 1e3
        comm_rest = 0.0 if P == 1 else c_rest * args.alpha_us * 1e-3 + b_rest / beta * 1e3
        row = {"P": P, "sweep_collectives": c_sw if P > 1 else 0, "sweep_recv_GB": b_sw / 1e9,
               "trtri_collectives": c_tr, "trtri_recv_GB": b_tr / 1e9,
               "comm_ms": comm_sweep + comm_tr + comm_rest,
               "comm_sweep_ms": comm_sweep, "comm_trtri_ms": comm_tr}
        if args.p1_ms and args.p1_value_ms:
            chain = nb * args.chain_us * 1e-3
            sweep = args.p1_value_ms
            grad = args.p1_ms - args.p1_value_ms
            bulk = max(0.0, sweep - chain)
            # the chain (factor, broadcast, panel, all-gather per step) does not divide; the
            # bulk does (taken as not overlapping the chain: at P = 1 this is the measurement)
            t_sweep = chain + comm_sweep + bulk / P
            row["predicted_ms"] = t_sweep + grad / P + comm_tr + comm_rest
            row["speedup_vs_p1"] = args.p1_ms / row["predicted_ms"]
        rows.append(row)
    for r in rows:
        print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()}))


if __name__ == "__main__":
    main()
