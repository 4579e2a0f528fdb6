#!/usr/bin/env python3
"""Memory-side traffic model of one k_bcr_split launch (what the EA counters see), beside the roofline's
algorithmic bytes (ba_solver.cpp K_BCR_PERSIST: S read once, each hand-off written once and read once).

The split kernel runs each 64-dof block on three workgroups (F factors D_i; helpers A / B carry the XL / XR
columns and x) and hands everything between workgroups through memory (ba_bcr.hip k_bcr_split):
  - F publishes its panels (lower L tiles, W_kb, 1/diag: 3648 doubles); both helpers read them
    (the root has helper B only);
  - at every survived level m of block i (neighbours a = i - 2^m, b = i + 2^m that exist), F pulls XR_a and
    XL_b (64 x 64 each), and each helper pulls XR_a, XL_b, x_a, x_b; at the block's last survived level
    helper A also pulls XL_a and helper B XR_b (the fills);
  - helper A publishes XL (if the block has a left neighbour at its own level) and x, helper B XR;
    helper B publishes y (back-substitution) and reads its two neighbours' y; the root reads every Gram;
  - every published slot of the next epoch is first written EMPTY (the flag-free protocol), so each
    published byte is written twice per launch.
Polls of slots that are still EMPTY are not modelled: each is one more 128-B line read.

usage: bcr_traffic_model.py [nblk=20] [measured_read_requests] [measured_write_requests]
(the elimination tree is the kernel's: virtual index v = i + voff, level ctz(v), root = block nblk / 2)"""
import sys

D = 8  # bytes per double
BSZ = 64 * 64 * D  # one published 64 x 64 row block set (XL or XR)
RSZ = 64 * 8 * D  # x / y slot (64 rows x 8 rhs columns)
PANEL = (10 * 256 + 4 * 256 + 64) * D  # lower tiles + W_0..3 + 1/diag


def tree(nblk):
    vl = 0
    while (2 << vl) <= nblk:
        vl += 1
    voff = (1 << vl) - nblk // 2
    root = nblk // 2

    def lvl(i):
        if i == root:
            return vl
        v = i + voff
        return (v & -v).bit_length() - 1

    return root, lvl


def model(nblk):
    root, lvl = tree(nblk)
    r = dict(s_inputs=0.0, panels=0.0, pulled_rows=0.0, y_and_gram=0.0)
    w = dict(panels=0.0, published_rows=0.0, y=0.0)
    for i in range(nblk):
        mi, is_root = lvl(i), i == root
        s_i = 1 << mi
        has_l = not is_root and i - s_i >= 0
        has_r = not is_root and i + s_i < nblk
        nh = 1 if is_root else 2
        # S inputs: D_i, the level-0 couplings (left / right), border rows, rhs (read once per block by its WGs)
        r["s_inputs"] += BSZ + (2 * BSZ if mi == 0 else 0) + 4 * 64 * D + RSZ
        for m in range(mi):
            s = 1 << m
            ha, hb = i - s >= 0, i + s < nblk
            last = m == mi - 1 and not is_root
            r["pulled_rows"] += (ha + hb) * BSZ  # F
            r["pulled_rows"] += nh * (ha + hb) * (BSZ + RSZ)  # helpers
            if last:
                r["pulled_rows"] += (has_l and ha) * BSZ + (has_r and hb) * BSZ  # fills
        r["panels"] += nh * PANEL
        w["panels"] += 2 * PANEL
        w["published_rows"] += 2 * (has_l * BSZ + has_r * BSZ + (has_l or has_r) * RSZ)
        w["y"] += 2 * RSZ
        r["y_and_gram"] += (has_l + has_r) * RSZ + (nblk * 25 * D if is_root else 0)
    return r, w


def main():
    nblk = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    r, w = model(nblk)
    rt, wt = sum(r.values()), sum(w.values())
    print(f"k_bcr_split traffic model, nblk = {nblk}")
    for k, v in r.items():
        print(f"  read  {k:<15} {v / 1e6:7.3f} MB")
    print(f"  read  total           {rt / 1e6:7.3f} MB = {rt / 128:9.0f} 128-B lines")
    for k, v in w.items():
        print(f"  write {k:<15} {v / 1e6:7.3f} MB")
    print(f"  write total           {wt / 1e6:7.3f} MB = {wt / 64:9.0f} 64-B requests")
    if len(sys.argv) > 3:
        mr, mw = float(sys.argv[2]), float(sys.argv[3])
        print(f"  measured: {mr:.0f} read requests x 128 B = {mr * 128 / 1e6:.3f} MB (model {rt / (mr * 128):.0%}), "
              f"{mw:.0f} write requests x 64 B = {mw * 64 / 1e6:.3f} MB (model {wt / (mw * 64):.0%})")
        print(f"  unmodelled reads (polls of EMPTY slots, partial lines): {(mr * 128 - rt) / 1e6:.3f} MB "
              f"= {(mr * 128 - rt) / 128:.0f} lines")


if __name__ == "__main__":
    main()
