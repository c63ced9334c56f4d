"""LDS bank-conflict model of fft_lds (lte_common.h) and the receivers' sample
loader (lte_dev.h load_symbol_noisy2), per element size.

Bank rules (MI355X_MICROARCH.md, LDS table): extra cycles per wave-instruction
= sum over the instruction's lane groups of (max distinct addresses on one bank
slot - 1).
  16-B elements: ds_read_b128 in the 16-lane groups {0-3,12-15,20-27},
  {4-11,16-19,28-31} (+32), banks (a/4) mod 64 -> element mod 16;
  ds_write_b128 in 8 x 8 contiguous lanes, banks (a/4) mod 32 -> element mod 8.
  8-B elements: ds_read_b64 in 2 x 32 lanes, element mod 32; ds_write_b64 in
  4 x 16 contiguous lanes, element mod 16.

Usage: python scripts/lds_bank_model.py   (prints extra cycles per instruction)
"""

RD16 = [[*range(0, 4), *range(12, 16), *range(20, 28)], [*range(4, 12), *range(16, 20), *range(28, 32)]]
RD16 += [[l + 32 for l in g] for g in RD16]
WR16 = [list(range(8 * k, 8 * k + 8)) for k in range(8)]
RD8 = [list(range(0, 32)), list(range(32, 64))]
WR8 = [list(range(16 * k, 16 * k + 16)) for k in range(4)]
RULES = {16: (RD16, 16, WR16, 8), 8: (RD8, 32, WR8, 16)}


def sw_f2(i):      # fft_sw<float2>
    return i ^ (((i >> 4) & 7) | ((i >> 3) & 8))


def sw_d2(i):      # fft_sw<double2>
    return i ^ ((i >> 3) & 7)


def ident(i):
    return i


def extra(addr, groups, mod):
    ex = 0
    for g in groups:
        slots = {}
        for lane in g:
            a = addr[lane]
            slots.setdefault(a % mod, set()).add(a)
        ex += max(len(v) for v in slots.values()) - 1
    return ex


def fft_model(esz, sw, N, isw=False):
    """Mean extra cycles per read / write instruction over every pass of one
    workgroup of 256 threads (N/8 threads per transform, 256/(N/8) transforms)."""
    rd_g, rd_m, wr_g, wr_m = RULES[esz]
    T = N // 8
    log2N = N.bit_length() - 1
    n8, rem = log2N // 3, log2N - 3 * (log2N // 3)
    lanes = range(256)
    slot = [l // T for l in lanes]
    jj = [l % T for l in lanes]
    rd = wr = nr = nw = 0

    def waves(f, groups, mod):
        tot = 0
        for w in range(4):
            tot += extra([f(l) for l in range(64 * w, 64 * w + 64)], groups, mod)
        return tot, 4

    Ns, lNs = 1, 0
    for s in range(n8):
        rsw = s > 0 or isw
        wsw = not (s == n8 - 1 and rem == 0)
        for r in range(8):
            t, n = waves(lambda l: slot[l] * N + (sw if rsw else ident)(jj[l] + r * T), rd_g, rd_m)
            rd += t; nr += n
            t, n = waves(lambda l: slot[l] * N + (sw if wsw else ident)(
                ((jj[l] >> lNs) << (lNs + 3)) + (jj[l] & (Ns - 1)) + r * Ns), wr_g, wr_m)
            wr += t; nw += n
        Ns <<= 3
        lNs += 3
    if rem:
        nb = 8 >> rem            # butterflies per thread (radix 4: 2, radix 2: 4)
        rad = 1 << rem
        step = N // rad
        for q in range(nb):
            for r in range(rad):
                t, n = waves(lambda l: slot[l] * N + sw(jj[l] + q * T + r * step), rd_g, rd_m)
                rd += t; nr += n
                t, n = waves(lambda l: slot[l] * N + jj[l] + q * T + r * step, wr_g, wr_m)
                wr += t; nw += n
    return rd / nr, wr / nw


def loader_model(esz, sw, N, off=144):
    """load_symbol_noisy2: lane t stores samples 2(p0 + t) - off and +1."""
    _, _, wr_g, wr_m = RULES[esz]
    T = N // 8
    p0 = off >> 1
    tot = n = 0
    for i in range(5):
        for c in (0, 1):
            addr = []
            for l in range(64):
                e = 2 * (p0 + l + i * T) + c - off
                addr.append(sw(e % N) if 0 <= e < N else 10 ** 6 + l)   # out-of-range lanes store nothing
            tot += extra(addr, wr_g, wr_m)
            n += 1
    return tot / n


if __name__ == '__main__':
    for N in (128, 256, 512, 1024, 2048):
        for esz, name, sw in ((8, 'float2', sw_f2), (16, 'double2', sw_d2), (16, 'double2 w/ float2 fold', sw_f2)):
            r, w = fft_model(esz, sw, N, isw=True)
            print(f"N={N:5d} {name:24s} fft read {r:.2f} write {w:.2f}  loader swizzled {loader_model(esz, sw, N):.2f}"
                  f"  loader natural {loader_model(esz, ident, N):.2f}")
