"""Exhaustive search for an XOR swizzle of 16-B chunks in a [rows][64] bf16 LDS image (128-B rows)
that is bank-conflict free for BOTH access patterns used by csrc/kernels/attention.hip:

* ds_read_b128 row reads: lane l reads row (l & 31) (+32·sub), chunk 2s + (l >> 5); lane groups per
  MI355X_MICROARCH.md §LDS ({0-3,12-15,20-27}, {4-11,16-19,28-31}, same +32);
* ds_read_b64_tr_b16 reads: per 32-lane half, 4 consecutive rows × 4 chunks × 2 eight-byte halves.

f(row) = XOR of per-bit 3-bit columns over row bits 1..5; the result printed is the column table.
Result (used in the kernel): f(row) = ((row>>1)&1)<<2 | ((row>>3)&3) — worst-case 1-way.
"""
import itertools

G128 = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
        list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
G128 = G128 + [[l + 32 for l in g] for g in G128]


def slot(row, c, f):
    return (row & 1) * 8 + (c ^ f(row))


def cost(f):
    worst, total = 0, 0
    for base in (0, 32):
        for s in range(4):
            for g in G128:
                slots = {}
                for l in g:
                    row, c = base + (l & 31), 2 * s + (l >> 5)
                    slots.setdefault(slot(row, c, f), set()).add((row, c))
                w = max(len(v) for v in slots.values())
                worst, total = max(worst, w), total + w
    for R in range(0, 64, 4):
        for dblk in (0, 1):
            slots = {}
            for dsub in (0, 1):
                for i in range(16):
                    row, c = R + (i >> 2), dblk * 4 + 2 * dsub + ((i & 3) >> 1)
                    slots.setdefault((slot(row, c, f), i & 1), set()).add((row, c))
            w = max(len(v) for v in slots.values())
            worst, total = max(worst, w), total + w
    return worst, total


def main():
    bits = [1, 2, 3, 4, 5]
    best = None
    for m in itertools.product(range(8), repeat=len(bits)):
        def f(row, m=m):
            v = 0
            for b, col in zip(bits, m):
                if (row >> b) & 1:
                    v ^= col
            return v
        c = cost(f)
        if best is None or c < best[0]:
            best = (c, m)
    print("unswizzled:", cost(lambda r: 0), " best:", best)


if __name__ == "__main__":
    main()
