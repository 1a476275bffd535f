"""LDS bank-conflict model of one Keccak round of grp_keccak16
(merlin_group.cuh) for two 16-lane groups sharing a 32-lane half, per the
gfx950 rule (cdna_hip_programming.md "Bank structure"): ds_read_b32 and
ds_write_b32 bank = dword address mod 32, serviced per 32-lane half, each
extra distinct address on a bank costs one LDS cycle; identical addresses
broadcast.  Prints the extra cycles per round (5 pi stores + 15 chi loads)
for the former layout and the best (trash base, group stride mod 32).

    python tools/lds_banks.py
"""
# rho offsets r[x][y], indexed [y][x] as GRP_RHO packs them
RHO = [[0, 1, 62, 28, 27], [36, 44, 6, 55, 20], [3, 10, 43, 25, 39], [41, 45, 15, 21, 8], [18, 2, 61, 56, 14]]


def store_addr(y, gl, trash):
    j, h = gl >> 1, gl & 1
    x = (j + 4) % 5
    n = RHO[y][x]
    s = n & 31
    sw = (n >> 5) ^ (1 if s == 0 else 0)
    Y = (2 * x + 3 * y) % 5
    return 2 * (5 * y + Y) + (sw ^ h) if 1 <= j <= 5 else trash + 2 * y + h


def load_addr(k, y, gl):
    j, h = gl >> 1, gl & 1
    x = (j + 4) % 5
    return 10 * ((x + k) % 5) + h + 2 * y


def extra(addrs):
    banks = {}
    for a in addrs:
        banks.setdefault(a % 32, set()).add(a)
    return max(len(v) for v in banks.values()) - 1


def round_cost(base0, base1, trash):
    st = ld = 0
    for y in range(5):
        st += extra([base0 + store_addr(y, l, trash) for l in range(16)] +
                    [base1 + store_addr(y, l, trash) for l in range(16)])
        for k in range(3):
            ld += extra([base0 + load_addr(k, y, l) for l in range(16)] + [base1 + load_addr(k, y, l) for l in range(16)])
    return st, ld


if __name__ == "__main__":
    print("former (scratch at 60 + 120 g dwords, trash 50):", round_cost(60, 180, 50))
    best = sorted((sum(round_cost(0, 96 + d, t)), t, d) for t in range(50, 80) for d in range(32))[:5]
    print("best (extra cycles, trash base, stride mod 32):", best)
    print("chosen (576-B stride = 144 dwords, trash 60):", round_cost(50, 50 + 144, 60))
