"""Bank-conflict check of fbank.hip's per-wave FFT buffer layout (development tool).

The buffer holds 256 complex f64 entries (16 B each, 16 slots per 256-B LDS row) at index
zsw(i) = i ^ (((i >> 4) & 1) * 13).  Lane groups per instruction (MI355X_MICROARCH.md §LDS):
ds_read_b128 serves {0-3, 12-15, 20-27}, {4-11, 16-19, 28-31} and the same + 32; ds_write_b128
serves 8 contiguous lanes.  A group costs one cycle per distinct address on its busiest
16-B slot.  Prints the extra cycles of every FFT access of one frame under the identity layout,
r5's first swizzle (XOR by 5 * ((i >> 4) & 3)) and the shipped one.

    python tools/fbank_banks.py
"""

READ_B128 = [list(range(0, 4)) + list(range(12, 16)) + list(range(20, 28)),
             list(range(4, 12)) + list(range(16, 20)) + list(range(28, 32))]
READ_B128 += [[l + 32 for l in g] for g in READ_B128]
WRITE_B128 = [list(range(8 * g, 8 * g + 8)) for g in range(8)]

LAYOUTS = {
    "identity": lambda i: i,
    "xor5*((i>>4)&3)": lambda i: i ^ (((i >> 4) & 3) * 5),
    "xor13*((i>>4)&1) (shipped)": lambda i: i ^ (((i >> 4) & 1) * 13),
}


def extra_cycles(groups, entry_of_lane, layout):
    extra = 0
    for g in groups:
        slots = {}
        for lane in g:
            e = layout(entry_of_lane(lane))
            slots.setdefault(e % 16, set()).add(e)
        extra += max(len(v) for v in slots.values()) - 1
    return extra


def accesses():
    """(name, kind, entry(lane)) of one frame: initial z writes (r5 keeps them in registers, listed
    for the layout comparison), Stockham stage reads / writes, the split's reads."""
    out = []
    for q in range(4):
        out.append((f"z write q={q}", "w", lambda l, q=q: l + 64 * q))
    for ns in (1, 4, 16, 64):
        for r in range(4):
            out.append((f"stage ns={ns} read r={r}", "r", lambda l, r=r: l + 64 * r))
        for m in range(4):
            out.append((f"stage ns={ns} write m={m}", "w",
                        lambda l, ns=ns, m=m: (l // ns) * ns * 4 + (l & (ns - 1)) + m * ns))
    for q in range(4):
        out.append((f"split read z q={q}", "r", lambda l, q=q: l + 64 * q))
        out.append((f"split read zc q={q}", "r", lambda l, q=q: (256 - (l + 64 * q)) & 255))
    return out


def main():
    for name, lay in LAYOUTS.items():
        assert sorted(lay(i) for i in range(256)) == list(range(256)), name
        tot, worst = 0, []
        for an, kind, ent in accesses():
            x = extra_cycles(READ_B128 if kind == "r" else WRITE_B128, ent, lay)
            tot += x
            if x:
                worst.append(f"{an}: +{x}")
        print(f"{name:28s} extra cycles per frame {tot:3d}   " + ", ".join(worst[:6]) + (" ..." if len(worst) > 6 else ""))


if __name__ == "__main__":
    main()
