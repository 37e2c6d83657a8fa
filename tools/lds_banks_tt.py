#!/usr/bin/env python3
"""LDS bank-conflict model of the TabTransformer block kernels' LDS accesses (csrc/tt_block.hip),
from the CDNA4 banking rules (/opt/skills/guides/MI355X_MICROARCH.md §LDS: per-instruction lane
groups, bank = (addr / 4) mod 64 for ds_read_b64 / b128 / tr_b16, mod 32 for b32 reads and every
write; one extra LDS cycle per extra distinct address on a bank within a group).

For each access pattern of the forward and backward kernels it counts, per wave instruction, the
conflict-free cycles and the extra cycles, weighted by how often a wave issues it per sample; then
it searches the row paddings (HS_LD fp32, AS_LD / QKV_LD / F_LD bf16) for the least extra cycles
within the LDS budget of two workgroups per CU.

    python tools/lds_banks_tt.py            # the current paddings and the best found
"""
import itertools

T, DM, FF, DH = 64, 64, 256, 16

GROUPS = {
    "b32r": [list(range(0, 32)), list(range(32, 64))],
    "b64r": [list(range(0, 32)), list(range(32, 64))],
    "b128r": [[*range(0, 4), *range(12, 16), *range(20, 28)], [*range(4, 12), *range(16, 20), *range(28, 32)],
              [*range(32, 36), *range(44, 48), *range(52, 60)], [*range(36, 44), *range(48, 52), *range(60, 64)]],
    "b32w": [list(range(0, 32)), list(range(32, 64))],
    "b64w": [list(range(16 * i, 16 * i + 16)) for i in range(4)],
    "b128w": [list(range(8 * i, 8 * i + 8)) for i in range(8)],
}
NBANK = {"b32r": 32, "b64r": 64, "b128r": 64, "b32w": 32, "b64w": 32, "b128w": 32}
WIDTH = {"b32r": 4, "b64r": 8, "b128r": 16, "b32w": 4, "b64w": 8, "b128w": 16}


def cycles(kind, addrs):
    """(conflict-free cycles, extra cycles) of one wave instruction; addrs[lane] = byte address."""
    nb, w = NBANK[kind], WIDTH[kind]
    extra = 0
    for grp in GROUPS[kind]:
        banks = {}
        for l in grp:
            a = addrs[l] - addrs[l] % 4 if w == 4 else addrs[l]
            for d in range(max(1, w // 4)):
                b = (a // 4 + d) % nb
                banks.setdefault(b, set()).add(a // 4 + d)
        extra += max(len(s) for s in banks.values()) - 1
    return len(GROUPS[kind]), extra


def patterns(HS_LD, AS_LD, QKV_LD, F_LD):
    """(name, kind, count per sample per wave, addr(lane, *it)) of the main LDS accesses."""
    HSB, ASB, QB, FB = HS_LD * 4, AS_LD * 2, QKV_LD * 2, F_LD * 2
    L = range(64)
    pats = []

    def add(name, kind, n, fn):
        pats.append((name, kind, n, [fn(l) for l in L]))

    for wv in range(1):  # wave 0 is representative (the others shift rows by 16 / columns by 16)
        # LayerNorm rows: lane -> row r = 16 wv + (l & 15), 16 floats at 16 g
        add("ln read HS (b128)", "b128r", 4 * 2, lambda l: (16 * wv + (l & 15)) * HSB + 64 * (l >> 4))
        add("ln write HS (b128)", "b128w", 4, lambda l: (16 * wv + (l & 15)) * HSB + 64 * (l >> 4))
        add("ln write AS (b128)", "b128w", 2 * 2, lambda l: (16 * wv + (l & 15)) * ASB + 32 * (l >> 4))
        # MFMA A fragments: row 16 i + c, 8 k at 32 ks + 8 g (bf16)
        add("A-frag AS/OS (b128)", "b128r", 4 * 2 * 3, lambda l: (l & 15) * ASB + 16 * (l >> 4))
        add("A-frag F (b128)", "b128r", 4 * 8, lambda l: (l & 15) * FB + 16 * (l >> 4))
        # QKV epilogue: 2-byte stores RS[(16 i + 4 g + r) * QKV_LD + t DM + DH wv + c]
        add("qkv store (b16)", "b32w", 3 * 4 * 4, lambda l: (4 * (l >> 4)) * QB + 2 * (DH * wv + (l & 15)))
        # attention: K / Q rows (b64), V column gathers (b16 reads)
        add("k/q frag (b64)", "b64r", 8, lambda l: (l & 15) * QB + 2 * DM + 2 * DH * wv + 8 * (l >> 4))
        add("v gather (b16)", "b32r", 16, lambda l: (4 * (l >> 4)) * QB + 2 * (2 * DM + DH * wv + (l & 15)))
        add("o store (b16)", "b32w", 16, lambda l: (4 * (l >> 4)) * ASB + 2 * (DH * wv + (l & 15)))
        # residual RMW: HS[(16 i + 4 g + r) * HS_LD + 16 wv + c]
        add("HS rmw read (b32)", "b32r", 2 * 16, lambda l: (4 * (l >> 4)) * HSB + 4 * (16 * wv + (l & 15)))
        add("HS rmw write (b32)", "b32w", 2 * 16, lambda l: (4 * (l >> 4)) * HSB + 4 * (16 * wv + (l & 15)))
        # fc1 epilogue: 8-byte stores of 4 consecutive columns of one token
        add("F store (b64)", "b64w", 16, lambda l: (l & 15) * FB + 2 * (64 * wv + 4 * (l >> 4)))
    return pats


def score(HS_LD, AS_LD, QKV_LD, F_LD, verbose=False):
    tot_base = tot_extra = 0
    for name, kind, n, addrs in patterns(HS_LD, AS_LD, QKV_LD, F_LD):
        base, extra = cycles(kind, addrs)
        tot_base += n * base
        tot_extra += n * extra
        if verbose:
            print(f"  {name:22s} {kind:6s} x{n:3d}: {base} + {extra} extra cycles per instruction")
    return tot_base, tot_extra


def lds_bytes(HS_LD, AS_LD, QKV_LD, F_LD):
    return T * HS_LD * 4 + 2 * T * AS_LD * 2 + T * max(F_LD, QKV_LD) * 2


def main():
    cur = (DM + 4, DM + 8, 3 * DM + 8, FF + 8)
    b, e = score(*cur, verbose=True)
    print(f"current {cur}: {b} conflict-free + {e} extra LDS cycles per wave per sample "
          f"({100 * e / (b + e):.1f} %), {lds_bytes(*cur)} B")
    best = None
    for hs in range(DM, DM + 33, 4):
        for asl in range(DM, DM + 49, 8):
            for q in range(3 * DM, 3 * DM + 49, 8):
                for f in range(FF, FF + 97, 8):
                    cfg = (hs, asl, q, f)
                    if 2 * lds_bytes(*cfg) > 160 * 1024:
                        continue
                    b2, e2 = score(*cfg)
                    key = (e2, lds_bytes(*cfg))
                    if best is None or key < best[0]:
                        best = (key, cfg)
    (e2, nbytes), cfg = best
    print(f"best {cfg}: {e2} extra cycles, {nbytes} B")
    score(*cfg, verbose=True)


if __name__ == "__main__":
    main()
