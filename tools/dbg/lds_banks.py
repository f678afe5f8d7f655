"""Bank model of the Winograd kernels' ds_read_b128 halo reads (gfx950).

ds_read_b128 serves a wave in four 16-lane groups — lanes {0-3, 12-15, 20-27}, {4-11, 16-19,
28-31} and the same +32 (MI355X_MICROARCH.md §LDS) — each group reading one 256-B bank row: it is
conflict-free iff its 16 lanes address 16 distinct 16-B slots (float4 index mod 16).  This
restates the halo layouts of conv_wino.h (WinoGeom) and conv_wino5.h (Wino5Geom) and prints, per
instantiated geometry, the worst slot multiplicity over the lane groups and tap offsets (1 =
conflict-free).  Layout constants here must match the headers.

usage: python tools/dbg/lds_banks.py
"""
import collections

GROUPS = ([0, 1, 2, 3, 12, 13, 14, 15] + list(range(20, 28)),
          list(range(4, 12)) + [16, 17, 18, 19] + list(range(28, 32)))


def worst(addr_of_lane, offsets):
    w = 1
    for off in offsets:
        for g in GROUPS:
            for hh in (0, 1):  # lanes +32: the second channel quad (+1 float4)
                c = collections.Counter((addr_of_lane(li) + hh + off) % 16 for li in g)
                w = max(w, max(c.values()))
    return w


def wino5(direction, W):
    """conv_wino5.h: 32 tiles of 4 pixels along the conv axis; 8 taps."""
    TPR = W // 4 if direction == 0 else 32
    OROWS = 128 // W if direction == 0 else 4
    HC = W + 4 if direction == 0 else 32
    SK = 4 if direction == 0 else 2
    ROWP = HC * 8 + HC // SK + (15 if direction == 0 else 0)

    def addr(r, c):
        return r * ROWP + c * 8 + c // SK

    def lane(li):
        return addr(li // TPR, 4 * (li % TPR)) if direction == 0 else addr(0, li)
    taps = [t * 8 + t // SK if direction == 0 else t * ROWP for t in range(8)]
    return worst(lane, taps), OROWS


def wino(W):
    """conv_wino.h: 32 2×2 tiles; the patch rows r1/r2 and columns b of each wave."""
    OCOLS = W if W < 64 else 64
    TW = OCOLS // 2
    HC = OCOLS + 2
    ROWP = HC * 8 + HC // 2 + (7 if TW < 32 else 0)

    def addr(r, c):
        return r * ROWP + c * 8 + (c >> 1)

    def lane(li):
        return addr(2 * (li // TW), 2 * (li % TW))
    offs = [r * ROWP + b * 8 + (b >> 1) for r in range(4) for b in range(4)]
    return worst(lane, offs)


def enc_conv(S, tc, tm, KW=3, new=True):
    """encoder.hip enc_conv_kernel A-fragment reads: 5 float4 per halo pixel (16 channels + 4),
    stride-2 skew of one float4 every 2 columns and the row pitch enc_row_pitch picks (new), or
    the round-4 layout (row pitch hc·5, no skew)."""
    hc = (tc - 1) * S + KW
    if new:
        a4 = lambda hr, c, rp: hr * rp + 5 * c + (c >> 1 if S == 2 else 0)  # noqa: E731
        base = a4(0, hc, 0)
        best = None
        for pad in range(16):  # enc_row_pitch: least conflicted of 16 pitches
            cost = sum(worst(lambda li, wm=wm, r=r: a4(((wm * tm // 2 + 32 * r + li) // tc) * S,
                                                      ((wm * tm // 2 + 32 * r + li) % tc) * S, base + pad),
                             [0]) for wm in (0, 1) for r in range(tm // 64))
            if best is None or cost < best[0]:
                best = (cost, base + pad)
        rp = best[1]
    else:
        a4 = lambda hr, c, rp: (hr * hc + c) * 5  # noqa: E731
        rp = 0
    return max(worst(lambda li, wm=wm, r=r: a4(((wm * tm // 2 + 32 * r + li) // tc) * S,
                                              ((wm * tm // 2 + 32 * r + li) % tc) * S, rp), [0])
               for wm in (0, 1) for r in range(tm // 64))


def lookup_tb(wp, dslot, D=9):
    """lookup.hip tile-row lookup, sampling phase: the 16 lanes of a pixel read sample s = 16j +
    lane's tap at row-major region offset b·wp + a (a, b = divmod(s, D)); ds_read_b32 serves 32
    lanes (two pixels, slot stride dslot floats) per pass over 32 banks.  Returns the summed
    worst multiplicity over the rounds (6 = conflict-free at D = 9)."""
    tot = 0
    for j in range((D * D + 15) // 16):
        addrs = [((b * wp + a) + pix * dslot) % 32 for pix in range(2) for gl in range(16)
                 for a, b in [divmod(16 * j + gl, D)] if 16 * j + gl < D * D]
        tot += max(collections.Counter(addrs).values())
    return tot


if __name__ == "__main__":
    for d in (0, 1):
        for W in (32, 64):
            print(f"conv_wino5_kernel DIR={d} W={W}: worst slot multiplicity {wino5(d, W)[0]}")
    for W in (32, 64, 128):
        print(f"conv_wino_kernel W={W}: worst slot multiplicity {wino(W)}")
    for S, tc, tm, what in ((2, 16, 64, "pose head conv 1 (32² -> 16²)"), (2, 8, 64, "pose head conv 2 (16² -> 8²)"),
                            (1, 128, 128, "encoder 3x3 s1 at 128²"), (2, 64, 128, "encoder 3x3 s2 -> 64²"),
                            (1, 16, 64, "encoder 3x3 s1 at 16²")):
        print(f"enc_conv_kernel S={S} tile {tm // tc}x{tc} ({what}): worst slot multiplicity "
              f"{enc_conv(S, tc, tm, new=False)} (round 4) -> {enc_conv(S, tc, tm)}")
    # tile-row lookup (r = 4): the layout in use (rows of 11 floats; two level regions per slot,
    # slot stride 2 · 124 + 4 = 252 floats) vs the best over row pitches 11..16 and slot strides
    cur = lookup_tb(11, 252 % 32)
    best = min((lookup_tb(wp, d), wp, d) for wp in range(11, 17) for d in range(32))
    print(f"corr_lookup_lds_kernel TB sampling: {cur} b32 passes per 6 rounds (ideal 6); best layout "
          f"{best[0]} at row pitch {best[1]}, slot stride ≡ {best[2]} mod 32")
