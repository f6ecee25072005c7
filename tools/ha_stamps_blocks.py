"""Per-block timelines of ha_step_kernel from MPGPU_HA_STAMPS=1 stamps (see tools/ha_stamps.py), for small
batches (the lone-scene tail): for a few stamped iterations, every block of scene 0 with its entry time and
phase stamps in us relative to the iteration's first block entry.

usage: python3 tools/ha_stamps_blocks.py stamps.bin [n_iterations]
slots: 0 entry, 1 body done (+ stores acknowledged), 2 role decided, 3 bookkeeping done, 4 finish done,
       nb groups 12 encode, 13 sweep, 14 need, 15 rs_heuristic, 16 end; RS block 12 search start,
       13 search end, 14 createActPath end, 16 end; bookkeeping 6 loads+dup, 7 FindNewNode, 10 pop scan
       loads, 11 pop reduce, 8 pop done."""
import sys

import numpy as np


def main(fn, n_it=6):
    raw = np.fromfile(fn, np.uint64)
    B, slots, nblk, every, ns = (int(x) for x in raw[:5].view(np.int64))
    st = raw[5:].reshape(slots, nblk, ns).astype(np.int64)
    tick = 0.01
    shown = 0
    for k in range(slots):
        e = st[k]
        used = e[:, 0] > 0
        if not (e[:, 1] > 0).any():
            continue
        t0 = e[used, 0].min()
        scene = (e[:, 5] >> 4) & 0xFFFFF
        item = e[:, 5] >> 32
        role = e[:, 5] & 0xF
        print(f"iteration {k * every}: blocks {int(used.sum())}")
        for b in np.nonzero(used & (scene == scene[used][0]))[0]:
            f = lambda j: f"{(e[b, j] - t0) * tick:5.1f}" if e[b, j] > 0 else "   - "
            kind = "RS " if item[b] == 0 else f"g{int(item[b]):02d}"
            line = f"  {kind} r{int(role[b])} entry {f(0)} | 12 {f(12)} 13 {f(13)} 14 {f(14)} 15 {f(15)} 16 {f(16)} | body {f(1)} role {f(2)}"
            if e[b, 3] == 0 and e[b, 6] > 0:  # (persistent tail, HA_SPEC) the runner-up job of an RS / group block
                line += f" | spec {f(6)} .. {f(7)}"
            if e[b, 3] > 0:
                line += f" | book: 6 {f(6)} 7 {f(7)} 10 {f(10)} 11 {f(11)} 8 {f(8)} done {f(3)}"
            if e[b, 4] > 0:
                line += f" | fin {f(4)}"
            print(line)
        shown += 1
        if shown >= n_it:
            break


if __name__ == "__main__":
    main(sys.argv[1], int(sys.argv[2]) if len(sys.argv) > 2 else 6)
