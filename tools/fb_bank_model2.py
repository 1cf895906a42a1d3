"""LDS bank-conflict model of the exact fbank's lane program with the
register post-pass (round 5, catears_amd/csrc/fbank8_ops.h): the phase-B
blocks are paired so that lane q holds the residue classes r and 16 - r of
the natural FFT index, the real-FFT post-pass takes both operands of every
pair from the lane's own registers, and LDS carries only the phase A -> B
transpose, the power spectrum and the mel reads.  Lane groups and bank
widths as tools/fb_bank_model.py (MI355X_MICROARCH.md, LDS).  Prints the
extra passes per 8-frame group (one wave) for frame strides S and
transpose layouts phys(p) = p + P * (p >> G), with the mel reads included.
python tools/fb_bank_model2.py"""
import math

from fb_bank_model import cost

kBlk1 = [0, 4, 10, 6, 14, 8, 12, 2]
kBlk2 = [1, 7, 13, 5, 9, 15, 11, 3]


def brev4(v):
    return ((v & 1) << 3) | ((v & 2) << 1) | ((v >> 1) & 2) | ((v >> 3) & 1)


R = [brev4(b) for b in kBlk1]  # class of block 1
assert sorted(R) == list(range(8)) and all((brev4(b2) + r) % 16 == 0 or (r == 0 and brev4(b2) == 8)
                                           for r, b2 in zip(R, kBlk2))


def mel_tables():
    lo = 1127 * math.log(1 + 20 / 700)
    hi = 1127 * math.log(1 + 8000 / 700)
    d = (hi - lo) / 41
    off, ln = [], []
    for b in range(40):
        left, right = lo + b * d, lo + (b + 2) * d
        bins = [k for k in range(256) if left < 1127 * math.log(1 + 31.25 * k / 700) < right]
        off.append(bins[0])
        ln.append(len(bins))
    W = [8, 12, 16, 24, 32]
    st = [[min(off[8 * c + q] & ~3, 256 - W[c]) for q in range(8)] for c in range(5)]
    return st, W


def model(S, P, G, mel=True):
    phys = lambda p: p + P * (p >> G)  # noqa: E731  (A -> B transpose only)
    fb = lambda l: (l >> 3) * S  # noqa: E731
    L = range(64)
    t = {}
    t['store_a'] = 2 * sum(cost([fb(l) + phys((l & 7) + 8 * j) for l in L], 'w32') for j in range(32))

    def pbp(q, j):
        return 16 * (kBlk1[q] if j < 16 else kBlk2[q]) + (j & 15)
    t['load_b'] = 2 * sum(cost([fb(l) + phys(pbp(l & 7, j)) for l in L], 'r128') for j in range(0, 32, 4))
    # power stores: per slot t two b32 stores (k side, partner side)
    A = [8 if q == 0 else R[q] for q in range(8)]
    C = [16 - R[q] for q in range(8)]
    D = [R[q] for q in range(8)]
    ps = 0
    for tt in range(16):
        c = brev4(tt)
        if c <= 7:
            k = [A[q] + 16 * c for q in range(8)]
        else:
            k = [C[q] + 16 * (15 - c) for q in range(8)]
        kk = [256 - x for x in k]
        ps += cost([fb(l) + kk[l & 7] for l in L], 'w32') + cost([fb(l) + k[l & 7] for l in L], 'w32')
    t['post_store'] = ps
    if mel:
        st, W = mel_tables()
        m = 0
        base = [0, 8, 20, 36, 60]
        for c in range(5):
            for i in range(0, W[c], 4):
                m += cost([fb(l) + st[c][l & 7] + i for l in L], 'r128')
                # weights: lane q's table at q * 92 + base[c] + i (shared by the 8 frames)
                m += cost([(l & 7) * 92 + base[c] + i for l in L], 'r128')
        t['mel'] = m
    return t


if __name__ == '__main__':
    res = []
    for S in range(256, 272, 4):
        for G in (4, 5, 6, 7):
            for P in (0, 4, 8):
                if 255 + P * (255 >> G) >= S:
                    continue
                tt = model(S, P, G)
                res.append((sum(tt.values()), S, P, G, tt))
    res.sort(key=lambda x: x[0])
    for r in res[:12]:
        print(r)
