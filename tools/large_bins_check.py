"""Which read-add-write batches of the large-window W-MSA backward's private CPB-gradient bins
are exact (wmsa_large.hip): with strided tiles on the lane (tile T = positions T + NT*li) and
contiguous 32-position chunks across the MFMA rows, count the batches in which two
(lane, element) pairs share a bin -- "query on the lane" (keys in the chunks) and "key on the
lane" (queries in the chunks, the binning phase since round 3).

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

        for phase in ("query on lane", "key on lane"):
            for name, size in (("chunk (8)", 8), ("half (4)", 4), ("element (1)", 1)):
                bad = tot = 0
                for tt in range(NT):
                    for c in range(NC):
                        for b0 in range(0, 8, size):
                            idx = []
                            for e in range(b0, b0 + size):
                                t, r = e >> 2, e & 3
                                for li in range(16):
                                    for g in range(4):
                                        m = 32 * c + 16 * t + 4 * g + r  # position in the chunk
                                        if m >= N:
                                            continue
                                        lanep = tt + NT * li
                                        idx.append(qb(lanep) - kb(m) if phase == "query on lane"
                                                   else qb(m) - kb(lanep))
                            tot += 1
                            bad += len(set(idx)) < len(idx)
                print(f"w{W} {phase}, batch {name}: {bad} of {tot} batches share a bin")


if __name__ == "__main__":
    main()
