"""LDS bank-conflict model for gfx950 (rules from the CDNA4 guide) used to pick GEMM swizzles."""
B128_GROUPS = [
    [0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27],
    [4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31],
]
B128_GROUPS += [[l + 32 for l in g] for g in B128_GROUPS]
HALF_GROUPS = [list(range(32)), list(range(32, 64))]


def cycles(addrs, groups, ndw):
    tot = 0
    for g in groups:
        banks = {}
        for l in g:
            a = addrs[l]
            for d in range(ndw):
                dw = a // 4 + d
                banks.setdefault(dw % 64, set()).add(dw)
        tot += max(len(s) for s in banks.values())
    return tot


def kmajor_read(swz, ks, base_row=0):
    # 16x16x32 A/B fragment from [row][64 bf16] (128 B rows); lane -> row l&15, chunk ks*4 + l>>4
    addrs = []
    for l in range(64):
        r = base_row + (l & 15)
        c = ks * 4 + (l >> 4)
        addrs.append(r * 128 + (c ^ swz(r)) * 16)
    return cycles(addrs, B128_GROUPS, 4)


def mnmajor_tr_read(swz, kstep, half, mn0):
    # ds_read_b64_tr_b16 from [k][128 bf16] (256 B rows): group g (16 lanes) reads rows
    # kstep*32 + 8g + 4*half + q (q=0..3), lane 4q+p -> cols mn0 + 4p .. +3
    addrs = []
    for l in range(64):
        g, i = l >> 4, l & 15
        q, p = i >> 2, i & 3
        k = kstep * 32 + 8 * g + 4 * half + q
        col = mn0 + 4 * p
        chunk, sub = col // 8, (col % 8) // 4
        addrs.append(k * 256 + (chunk ^ swz(k)) * 16 + sub * 8)
    return cycles(addrs, HALF_GROUPS, 2)


if __name__ == "__main__":
    km = {"none": lambda r: 0, "r&7": lambda r: r & 7, "(r>>1)&7": lambda r: (r >> 1) & 7,
          "r&7^r>>3": lambda r: (r & 7) ^ ((r >> 3) & 7)}
    for n, f in km.items():
        print("kmajor", n, [kmajor_read(f, ks, br) for ks in (0, 1) for br in (0, 16, 32)])
    mm = {"none": lambda k: 0,
          "even(k&3|k>>1&4)": lambda k: ((k & 3) | ((k >> 1) & 4)) << 1,
          "k&15": lambda k: k & 15,
          "k&7": lambda k: k & 7}
    for n, f in mm.items():
        print("mnmajor", n, [mnmajor_tr_read(f, ks, h, mn0) for ks in (0, 1) for h in (0, 1)
                             for mn0 in (0, 16, 48, 112)])
