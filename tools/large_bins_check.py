"""Which read-add-write batches of the large-window W-MSA backward's private CPB-gradient bins
are exact (wmsa_large.hip, loop B): with strided query tiles (query tile qt = positions
qt + NT*li), count the batches in which two (lane, element) pairs share a bin.

    python tools/large_bins_check.py"""


def main():
    for W in (12, 16, 24):
        N, R = W * W, 2 * W - 1
        NT, NC = N // 16, (N // 16 + 1) // 2

        def qb(p):
            y, x = divmod(p, W)
            return (y + W - 1) * R + x + W - 1

        def kb(p):
            y, x = divmod(p, W)
            return y * R + x

        for name, size in (("chunk (8)", 8), ("half (4)", 4), ("element (1)", 1)):
            bad = tot = 0
            for qt in range(NT):
                for c in range(NC):
                    for b0 in range(0, 8, size):
                        idx = []
                        for e in range(b0, b0 + size):
                            t, r = e >> 2, e & 3
                            for li in range(16):
                                for g in range(4):
                                    k = 32 * c + 16 * t + 4 * g + r
                                    if k < N:
                                        idx.append(qb(qt + NT * li) - kb(k))
                        tot += 1
                        bad += len(set(idx)) < len(idx)
            print(f"w{W} batch {name}: {bad} of {tot} batches share a bin")


if __name__ == "__main__":
    main()
