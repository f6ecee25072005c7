"""Per-iteration summary of ha_step_kernel stamps (MPGPU_HA_STAMPS=1, see tools/ha_stamps_blocks.py) for wide
batches: for every stamped iteration the blocks launched, the dispatch spread (last block entry - first), the
iteration span (last finish - first entry), and median / max durations of the RS_connected blocks' phases
(search, createActPath), the neighbour groups' phases (encode, sweep, rs_heuristic, whole body) and the
bookkeeping, in us (ha_pipe_kernel launches: the bookkeeping block's publish and done times from its entry;
the groups' encode phase then includes their wait for the publish).

usage: python3 tools/ha_stamps_wide.py stamps.bin"""
import sys

import numpy as np


def main(fn):
    raw = np.fromfile(fn, np.uint64)
    B, slots, nblk, every, ns = (int(x) for x in raw[:5].view(np.int64))
    st = raw[5:].reshape(slots, nblk, ns).astype(np.int64)
    tick = 0.01

    def md(x):
        x = np.asarray(x, float) * tick
        return f"{np.median(x):5.1f}/{x.max():5.1f}" if len(x) else "   -  /  -  "

    print("iter blocks  spread   span | RS search  RS path   RS body | g encode  g sweep   g rsh     g body  | book")
    for k in range(slots):
        e = st[k]
        used = (e[:, 0] > 0) & (e[:, 1] > 0)
        if not used.any():
            continue
        e = e[used]
        t0 = e[:, 0].min()
        item = e[:, 5] >> 32
        rs = item == 0
        g = (item >= 1) & (item < 17)
        pb = (item == 17) & (e[:, 8] > 0)  # ha_pipe_kernel's bookkeeping block
        ends = np.maximum.reduce([e[:, 1], e[:, 3], e[:, 4]])
        ok = lambda m, a, b: m & (e[:, a] > 0) & (e[:, b] > 0)
        rs_s = ok(rs, 13, 12)
        rs_p = ok(rs, 14, 13)
        g_e = ok(g, 12, 0)
        g_s = ok(g, 13, 12)
        g_r = ok(g, 15, 14)
        bk = (e[:, 3] > 0) & (e[:, 2] > 0) & ~pb
        print(f"{k * every:4d} {int(used.sum()):6d} {(e[:, 0].max() - t0) * tick:7.1f} {(ends.max() - t0) * tick:6.1f} | "
              f"{md(e[rs_s, 13] - e[rs_s, 12])} {md(e[rs_p, 14] - e[rs_p, 13])} {md(e[rs, 1] - e[rs, 0])} | "
              f"{md(e[g_e, 12] - e[g_e, 0])} {md(e[g_s, 13] - e[g_s, 12])} {md(e[g_r, 15] - e[g_r, 14])} "
              f"{md(e[g, 1] - e[g, 0])} | {md(e[bk, 3] - e[bk, 2])}" +
              (f" | pipe book: publish {md(e[pb, 8] - e[pb, 0])} done {md(e[pb, 3] - e[pb, 0])}" if pb.any() else ""))


if __name__ == "__main__":
    main(sys.argv[1])
