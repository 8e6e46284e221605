"""Predicted strong-scaling curve of the row-block objective (dev tool).

  python tools/dist_model.py --p1-ms MS --p1-value-ms MS [--points 16384] [--basis 11]
                             [--dims 10] [--widths 8:160,4:0] [--chain-us 90]

Counts, from the schedule of gpemu_dist.hip (column groups, recursive TRTRI chunks), the
collectives one LLH + gradient issues and the bytes each rank receives in them, then
predicts the evaluation time at P ranks over xGMI as

  T(P) = chain + sweep_bulk / P + (trtri + slab + rest) / P
         + sum over collectives of (alpha + received bytes / beta)

with the compute terms from the P = 1 loopback run (one GPU, no real collectives) and
alpha / beta the per-collective latency and per-rank receive bandwidth of RCCL over the
MI355X's xGMI (defaults: 25 us, 64 GB/s at P = 2 over one link, 300 GB/s at P >= 4).
The sweep's collectives sit on the chain (the look-ahead overlaps the bulk, not them).
Round 5 schedule: per column step ONE broadcast of [-M | Dinv] from the diagonal owner
(128 x 128 (1 + h) doubles at position h of its group), per column GROUP one all-gather of
the group's columns on the rows below it.  Also the per-rank device memory (the
allocations of gpe_dist_set_data / ensure_grad, descriptors left out)."""
import argparse
import json

TILE = 128
T2B = TILE * TILE * 8      # bytes per tile
SLAB_DOUBLES = 1 << 26


def nloc_of(nb, P, r):
    return (nb - r) // P + 1 if r <= nb else 0


def li0_of(k, P, r):
    return 0 if k < r else (k - r) // P + 1


def groups(nb, widths):
    gs, g = [], 0
    while g < nb:
        gs.append(g)
        w = next((a for a, m in widths if nb - g > m), 1)
        g += max(1, min(w, nb - g))
    gs.append(nb)
    return gs


def sweep_collectives(nb, na, P, widths):
    """(count, bytes received per rank): a broadcast per step, an all-gather per group."""
    nt = nb + na
    cnt, rb = 0, 0
    gs = groups(nb, widths)
    for g in range(len(gs) - 1):
        gb, ge = gs[g], gs[g + 1]
        for k in range(gb, ge):
            cnt += 1
            rb += T2B * (1 + k - gb) if P > 1 else 0                 # [-M | Dinv] from its owner
        T = max(max(0, nloc_of(nt - 1, P, r) - li0_of(ge - 1, P, r)) for r in range(P))
        if T > 0:
            cnt += 1
            rb += (P - 1) * T * (ge - gb) * T2B                     # all-gather (padded segments)
    return cnt, rb


def trtri_levels(nb, P, cap):
    """Per level (s, chunk width, g1, s1, g2, s2) of the recursive TRTRI, as ensure_grad."""
    out = []
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
        out.append((s, cc, g1, s1, g2, s2, pairs))
        s *= 2
    return out


def slab_doubles(nb, n_pad, P):
    whole = nb * TILE * n_pad
    sd = SLAB_DOUBLES
    if whole <= 4 * SLAB_DOUBLES:
        sd = max(sd, whole // P)
    return max(1, min(nb, sd // (TILE * n_pad))) * TILE * n_pad


def trtri_collectives(nb, P, cap):
    """(count, bytes received per rank) of the recursive TRTRI's chunked all-gathers."""
    cnt, rb = 0, 0
    for (s, cc, g1, s1, g2, s2, pairs) in trtri_levels(nb, P, cap * 8):
        a = s // 2
        for j0 in range(0, a, cc):
            cw, rows1 = min(cc, a - j0), a - j0
            seg1 = sum(-(-rows1 // P) * cw for _ in pairs)
            seg2 = sum(cw * -(-(t1 - h) // P) for (_, h, t1) in pairs)
            if P > 1:
                cnt += 2
                rb += (P - 1) * (seg1 + seg2) * T2B
    return cnt, rb


def rank_memory_gb(nb, na, P, d, pc, widths, grad=True, int8=True):
    """Device bytes of rank 0 (the largest share), in GB."""
    nt, n_pad = nb + na, nb * TILE
    gs = groups(nb, widths)
    wmax = max(gs[i + 1] - gs[i] for i in range(len(gs) - 1))
    nloc = nloc_of(nt - 1, P, 0)
    ld = max(nloc, 1) * TILE
    b = ld * nt * TILE + (nb + 1) + TILE * TILE * wmax + pc * pc       # A rows, logdet, [-M|Dinv], Gram
    recv = 0
    if P > 1:
        rt = max(max(max(0, nloc_of(nt - 1, P, r) - li0_of(gs[g + 1] - 1, P, r)) for r in range(P))
                 * (gs[g + 1] - gs[g]) for g in range(len(gs) - 1))
        recv = P * rt * TILE * TILE
        b += 2 * nt * TILE * TILE * wmax + recv                          # panels, all-gather buffer
    shared = n_pad * (2 * d + pc + 2) + nb * (nb + 1) // 2 * (d + 3)    # inputs, contraction partials
    if grad:
        sd = slab_doubles(nb, n_pad, P)
        b += ld * nb * TILE + 2 * n_pad * pc + ld * na * TILE + n_pad * na * TILE + sd + d + 3
        if P > 1:
            g1n = rvn = 0
            for (s, cc, g1, s1, g2, s2, pairs) in trtri_levels(nb, P, sd * 8):
                g1n = max(g1n, g1 * cc * TILE * TILE)
                rvn = max(rvn, P * s1 * cc * TILE * TILE, P * s2 * cc * TILE * TILE)
            b += g1n + (0 if rvn <= recv else rvn)
        # the int8 partial's planes and residues (gpemu_dist.hip oz_prepare; bytes), while the
        # planes fit 16 GiB
        np2 = -(-n_pad // 256) * 256
        kp = ((nb - 1) // P + 1) * TILE
        if int8 and 16 * np2 * kp <= 16 << 30:
            sr = max(1, min(nb, sd // (TILE * n_pad)))
            if sr < nb and sr % 2:
                sr = max(2, sr - 1)
            tri = lambda t: t * (t + 1) // 2
            maxt = max(tri((min(nb, a0 + sr) + 1) // 2) - tri(a0 // 2) for a0 in range(0, nb, sr))
            b += (16 * np2 * kp + 16 * maxt * 256 * 256) / 8
    return (b + shared) * 8 / 1e9


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--points", type=int, default=16384)
    ap.add_argument("--basis", type=int, default=11, help="q + 1")
    ap.add_argument("--dims", type=int, default=10)
    ap.add_argument("--widths", default="8:160,4:0", help="the row-block path's column-group widths")
    ap.add_argument("--p1-ms", type=float, default=None, help="loopback P=1 LLH+gradient ms")
    ap.add_argument("--p1-value-ms", type=float, default=None, help="loopback P=1 value-only ms")
    ap.add_argument("--chain-us", type=float, default=75.0, help="diagonal factor + panel per step, us")
    ap.add_argument("--alpha-us", type=float, default=25.0)
    ap.add_argument("--beta2", type=float, default=64.0, help="GB/s per rank at P=2")
    ap.add_argument("--beta", type=float, default=300.0, help="GB/s per rank at P>=4")
    ap.add_argument("--single-ms", type=float, default=None, help="the single-GPU path's LLH+gradient ms")
    ap.add_argument("--no-int8", action="store_true", help="memory without the int8 partial's buffers")
    ap.add_argument("--trtri-overlap", choices=("none", "prev-level", "full"), default="none",
                    help="TRTRI all-gathers hidden behind compute: none (round 5, in series), prev-level "
                         "(level l's gathers beside level l-1's products: round-6 verdict option 1), full "
                         "(a ring pass of X row blocks beside the products: option 2, upper bound)")
    args = ap.parse_args()
    widths = [tuple(int(v) for v in e.split(":")) for e in args.widths.split(",")]
    nb = -(-args.points // TILE)
    na = -(-args.basis // TILE)
    n_pad = nb * TILE
    rows = []
    for P in (1, 2, 4, 8):
        cap = slab_doubles(nb, n_pad, P)
        c_sw, b_sw = sweep_collectives(nb, na, P, widths)
        c_tr, b_tr = trtri_collectives(nb, P, cap)
        c_rest = 6                                                  # Gram, logdet, info, Z, W, sums
        b_rest = (P - 1) / P * (n_pad * args.basis * 8 * 2) if P > 1 else 0
        beta = (args.beta2 if P == 2 else args.beta) * 1e9
        comm_sweep = 0.0 if P == 1 else c_sw * args.alpha_us * 1e-3 + b_sw / beta * 1e3
        comm_tr = 0.0 if P == 1 else c_tr * args.alpha_us * 1e-3 + b_tr / beta * 1e3
        comm_rest = 0.0 if P == 1 else c_rest * args.alpha_us * 1e-3 + b_rest / beta * 1e3
        row = {"P": P, "sweep_collectives": c_sw if P > 1 else 0, "sweep_recv_GB": b_sw / 1e9,
               "trtri_collectives": c_tr, "trtri_recv_GB": b_tr / 1e9,
               "comm_ms": comm_sweep + comm_tr + comm_rest,
               "comm_sweep_ms": comm_sweep, "comm_trtri_ms": comm_tr,
               "rank_memory_GB": rank_memory_gb(nb, na, P, args.dims, args.basis, widths, int8=not args.no_int8)}
        if args.p1_ms and args.p1_value_ms:
            chain = nb * args.chain_us * 1e-3
            sweep = args.p1_value_ms
            grad = args.p1_ms - args.p1_value_ms
            bulk = max(0.0, sweep - chain)
            # the chain (factor, broadcast, panel per step; the group all-gathers) does not
            # divide; the bulk does (taken as not overlapping the chain: at P = 1 this is the
            # measurement)
            t_sweep = chain + comm_sweep + bulk / P
            t_grad = grad / P + comm_tr
            if P > 1 and args.trtri_overlap != "none":
                # per level: its products' share of the gradient compute (n S^2 of n^3 / 3 for the
                # TRTRI's 1 / 2 of it) and its gathers' time
                lv = trtri_levels(nb, P, cap * 8)
                tot = sum(s_ * s_ for (s_, *_r) in lv)
                trtri_ms = (grad / P) * 0.5
                comp = [trtri_ms * (s_ * s_) / tot for (s_, *_r) in lv]
                gath = []
                for (s_, cc, g1, s1, g2, s2, pairs) in lv:
                    a = s_ // 2
                    b = 0
                    for j0 in range(0, a, cc):
                        cw, rows1 = min(cc, a - j0), a - j0
                        b += (P - 1) * (sum(-(-rows1 // P) * cw for _ in pairs) +
                                        sum(cw * -(-(t1 - h) // P) for (_, h, t1) in pairs)) * T2B
                    gath.append(b / beta * 1e3 + 2 * args.alpha_us * 1e-3 * (-(-a // cc)))
                if args.trtri_overlap == "prev-level":
                    hidden = sum(min(gath[i], comp[i - 1]) for i in range(1, len(lv)))
                else:
                    hidden = min(sum(gath), grad / P)
                t_grad = grad / P + comm_tr - hidden
                row["trtri_comm_hidden_ms"] = hidden
            row["predicted_ms"] = t_sweep + t_grad + comm_rest
            row["speedup_vs_p1"] = args.p1_ms / row["predicted_ms"]
            if args.single_ms:
                row["speedup_vs_single_gpu"] = args.single_ms / row["predicted_ms"]
        rows.append(row)
    for r in rows:
        print(json.dumps({k: (round(v, 3) if isinstance(v, float) else v) for k, v in r.items()}))


if __name__ == "__main__":
    main()
