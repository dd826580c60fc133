"""LDS bank check of wgrad_halo's ds_read_b64_tr_b16 fragment reads (stride 1), per row width.

A tr read is serviced in two 32-lane halves; each half reads 8 LDS rows of 128 B (one pixel each), 32 B
per row, at 8-B units (unit ^ f(row)) << 3 with f = the row's 16-B chunk swizzle. The 8 rows hit 8 distinct
32-B bank slots -- conflict-free -- iff their (row parity, f(row)) pairs are distinct. The halo (x) side
reads every tap shift r * (W + 2) + s of the same 8 pixels; the dy side reads the pixel rows themselves.

For a pixel map (which pixel each (k-step, lane block, read, lane quad) reads; wg_pixel in wgrad_halo.hip)
and swizzle bits, prints the worst rows-per-slot over all taps, k-steps and halves for W = 32, 16, 8, 4
(1 = conflict-free). pmap 0 with row bits (1, 3) is the original layout; pmap 1 / 2 with the bits the
kernel uses for them (HaloParams::pmap) are conflict-free everywhere.
usage: python tools/tr_banks.py
"""


def wg_pixel(pmap, ks, b, h, q):
    if pmap == 1:
        return ks * 32 + 16 * h + 4 * b + q
    if pmap == 2:
        return ks * 32 + (b >> 1) * 16 + (h + 2 * (b & 1)) * 4 + q
    return ks * 32 + 8 * b + q + 4 * h


def geometry(W):
    H = W
    rs, imgs = (64 // W, 1) if H * W >= 64 else (H, 64 // (H * W))
    return W + 2, (rs + 2) * (W + 2), rs * W  # pitch, halo rows per image block, pixels per block


def halo_row(t, W):
    pitch, hb, spi = geometry(W)
    ii, rem = divmod(t, spi)
    pr, q = divmod(rem, W)
    return ii * hb + pr * pitch + q


def worst(rows, sb):
    slots = {}
    for r in rows:
        slots.setdefault((r & 1, ((r >> 1) & 1) | (((r >> sb) & 1) << 1)), set()).add(r)
    return max(len(v) for v in slots.values())


def check(W, pmap, hsb, dsb):
    pitch = W + 2
    wh = wd = 1
    for ks in range(2):
        for half in range(2):
            for h in range(2):
                pix = [wg_pixel(pmap, ks, b, h, q) for b in (2 * half, 2 * half + 1) for q in range(4)]
                wd = max(wd, worst(pix, dsb))
                base = [halo_row(t, W) for t in pix]
                for tap in range(9):
                    toff = (tap // 3) * pitch + tap % 3
                    wh = max(wh, worst([r + toff for r in base], hsb))
    return wh, wd


if __name__ == "__main__":
    layouts = {"pmap 0, bits (1,3) [original]": (0, 3, 3), "pmap 1, bits (1,2)": (1, 2, 2),
               "pmap 2, halo (1,2), dy (1,3)": (2, 2, 3)}
    for name, (pm, hsb, dsb) in layouts.items():
        print(name, {W: check(W, pm, hsb, dsb) for W in (32, 16, 8, 4) if not (pm == 2 and W != 4)})
