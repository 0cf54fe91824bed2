"""LDS bank check of pos_conv.hip's A-fragment reads (development tool, CPU only).

Lane l of a 16x16x32 step reads 16 B at patch byte 96 (32 w + 16 i + (l & 15)) + 2 (32 s + 8 (l >> 4))
(96-B rows: 48 bf16 channels, k = tap * 48 + c).  ds_read_b128 serves 4 lane groups of 16
(MI355X_MICROARCH.md §LDS); a group costs one LDS cycle per distinct address on its busiest 16-B slot
of the 256-B bank row.  Prints the worst and mean cycles per group over every k-step, wave and i
for a few row strides (in 16-B slots)."""
G = [[*range(0, 4), *range(12, 16), *range(20, 28)], [*range(4, 12), *range(16, 20), *range(28, 32)]]
G += [[l + 32 for l in g] for g in G]


def cost(sigma):
    tot = n = worst = 0
    for s in range(192):
        for w in range(8):
            for i in range(2):
                for g in G:
                    cnt = {}
                    for l in g:
                        kg = 32 * s + 8 * (l >> 4)
                        row = 32 * w + 16 * i + (l & 15) + kg // 48
                        slot = (row * sigma + (kg % 48) // 8) % 16
                        cnt[slot] = cnt.get(slot, 0) + 1
                    m = max(cnt.values())
                    tot, n, worst = tot + m, n + 1, max(worst, m)
    return worst, tot / n


if __name__ == "__main__":
    for sigma in (6, 7, 8, 9, 10):
        w, m = cost(sigma)
        print(f"row stride {16 * sigma:3d} B: worst {w} cycles / lane group, mean {m:.3f}")
