"""Phase timing of ha_step_kernel from MPGPU_HA_STAMPS=1 stamps (s_memrealtime, 100 MHz).

usage: (a library built with -DHA_STAMP_CODE=1) MPGPU_HA_STAMPS=1 MPGPU_HA_STAMPS_OUT=gpurun_out/ha_stamps.bin python3 tools/ha_plan_time.py
       python3 tools/ha_stamps.py gpurun_out/ha_stamps.bin
For every stamped iteration: the kernel span (first entry to last finish), and per scene the RS_connected
block's body, the neighbour groups' bodies (last one), the bookkeeping and the finisher, in us relative
to the iteration's first block entry; medians over scenes, then the critical scene.
"""
import sys

import numpy as np


def main(fn):
    raw = np.fromfile(fn, np.uint64)
    B, slots, nblk, every, ns = (int(x) for x in raw[:5].view(np.int64))
    st = raw[5:].reshape(slots, nblk, ns).astype(np.int64)
    tick = 0.01  # us per s_memrealtime tick (100 MHz)
    print(f"B={B} stamped iterations every {every}")
    print(f"{'it':>5} {'blocks':>6} {'span':>7} {'rs_body':>8} {'nb_body':>8} {'book':>7} {'finish':>7} | critical scene: rs nb book fin")
    for k in range(slots):
        e = st[k]
        used = e[:, 0] > 0
        done = e[:, 1] > 0
        if not done.any():
            continue
        t0 = e[used, 0].min()
        tl = lambda v: (v - t0) * tick
        role = e[:, 5] & 0xF
        scene = (e[:, 5] >> 4) & 0xFFFFF
        item = e[:, 5] >> 32
        rows = {}
        for b in np.nonzero(done)[0]:
            s = int(scene[b])
            r = rows.setdefault(s, {"rs": 0.0, "nb": 0.0, "book": 0.0, "fin": 0.0})
            if item[b] == 0:
                r["rs"] = tl(e[b, 1])
            else:
                r["nb"] = max(r["nb"], tl(e[b, 1]))
            if e[b, 3] > 0:
                r["book"] = tl(e[b, 3])
            if e[b, 4] > 0:
                r["fin"] = tl(e[b, 4])
        fin = np.array([r["fin"] for r in rows.values()])
        crit = max(rows.values(), key=lambda r: r["fin"])
        med = {key: np.median([r[key] for r in rows.values()]) for key in ("rs", "nb", "book", "fin")}
        span = fin.max()
        bk = np.nonzero(e[:, 3] > 0)[0]
        ph = ""
        if len(bk) and ns >= 10:
            d = lambda a, b_: np.median((e[bk, b_] - e[bk, a]) * tick)
            ph = (f" | book phases: role {d(1, 2):.1f} loads+dup {d(2, 6):.1f} FindNewNode {d(6, 7):.1f} "
                  f"pop {d(7, 8):.1f} record {d(8, 3):.1f}; n_open {int(np.median(e[bk, 9]))}")
            if ns >= 12:
                ph += f" | pop: loads {d(7, 10):.1f} reduce+barrier {d(10, 11):.1f} final+stores {d(11, 8):.1f}"
        if ns >= 17:  # block body phases from the block's entry (medians): nb 12 encode, 13 sweep, 14 need
            # barrier, 15 search, 16 end; RS 12 search start, 13 search end, 14 createActPath, 16 end
            nbb = np.nonzero(done & (item > 0))[0]
            rsb = np.nonzero(done & (item == 0))[0]
            md = lambda ix, j: np.median((e[ix, j] - e[ix, 0]) * tick) if len(ix) and (e[ix, j] > 0).all() else float("nan")
            ph += (f" | nb: encode {md(nbb, 12):.1f} sweep {md(nbb, 13):.1f} need {md(nbb, 14):.1f} "
                   f"end {md(nbb, 16):.1f}; rs: search {md(rsb, 12):.1f}-{md(rsb, 13):.1f} path {md(rsb, 14):.1f} "
                   f"end {md(rsb, 16):.1f}")
        print(f"{k * every:5d} {int(done.sum()):6d} {span:7.1f} {med['rs']:8.1f} {med['nb']:8.1f} {med['book']:7.1f} "
              f"{med['fin']:7.1f} | {crit['rs']:.1f} {crit['nb']:.1f} {crit['book']:.1f} {crit['fin']:.1f}{ph}")


if __name__ == "__main__":
    main(sys.argv[1])
