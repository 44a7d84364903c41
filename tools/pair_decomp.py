"""Search behind round 5's four-wave Correlation layout (measured and dropped, profiles/r5_ab.txt): four placements
of one 7-edge pattern on 6 positions that cover every pair of 8 columns exactly once, with two positions that
together hold every column once (the fused column moments).  Prints the first layout found per pattern class
(none exists on 5 positions)."""
import itertools
import sys
import time

EID = {e: i for i, e in enumerate(itertools.combinations(range(8), 2))}
FULL = (1 << 28) - 1
V = 6


def canon(es):
    return min(tuple(sorted(tuple(sorted((p[a], p[b]))) for a, b in es)) for p in itertools.permutations(range(V)))


def main():
    classes = {}
    for es in itertools.combinations(list(itertools.combinations(range(V), 2)), 7):
        if len({v for e in es for v in e}) == V:
            classes.setdefault(canon(es), es)
    for pat in classes.values():
        embs = {}
        for perm in itertools.permutations(range(8), V):
            m = 0
            for a, b in pat:
                x, y = perm[a], perm[b]
                m |= 1 << EID[(min(x, y), max(x, y))]
            embs.setdefault(m, perm)
        by_bit = [[] for _ in range(28)]
        for m, perm in embs.items():
            for b in range(28):
                if m >> b & 1:
                    by_bit[b].append((m, perm))
        found, t0 = [], time.time()

        def bt(cov, sol):
            if time.time() - t0 > 5:
                return True
            if cov == FULL:
                for p, q in itertools.combinations(range(V), 2):
                    if sorted(c for perm in sol for c in (perm[p], perm[q])) == list(range(8)):
                        found.append((p, q, list(sol)))
                        return True
                return False
            b = ((~cov) & FULL & -((~cov) & FULL)).bit_length() - 1
            for m, perm in by_bit[b]:
                if not m & cov:
                    sol.append(perm)
                    if bt(cov | m, sol):
                        return True
                    sol.pop()
            return False

        bt(0, [])
        if found:
            print("pattern", pat, "moments at", found[0][:2], "waves", found[0][2])
            sys.stdout.flush()


if __name__ == "__main__":
    main()
