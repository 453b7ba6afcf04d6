"""Rough VGPR pressure along a kernel's assembly (straight-line approximation: a register is live
from a definition to its last textual use; branches and loops ignored). Diagnostic only.

  python tools/vlive.py file.s kernel_symbol_prefix [window]
"""
import re
import sys

STORE_LIKE = ("ds_write", "ds_store", "buffer_store", "global_store", "scratch_store", "flat_store",
              "s_", "v_cmp", "v_cmpx", "ds_add", "ds_or", "global_atomic", "buffer_atomic")
REG = re.compile(r"\bv\[(\d+):(\d+)\]|\bv(\d+)\b|\ba\[(\d+):(\d+)\]|\ba(\d+)\b")


def regs(tok):
    out = []
    for m in REG.finditer(tok):
        if m.group(1):
            out += [("v", i) for i in range(int(m.group(1)), int(m.group(2)) + 1)]
        elif m.group(3):
            out.append(("v", int(m.group(3))))
        elif m.group(4):
            out += [("a", i) for i in range(int(m.group(4)), int(m.group(5)) + 1)]
        elif m.group(6):
            out.append(("a", int(m.group(6))))
    return out


def main(path, sym, window=40):
    lines, on = [], False
    for ln in open(path):
        if ln.startswith(sym):
            on = True
        if on:
            lines.append(ln.rstrip("\n"))
            if "s_endpgm" in ln:
                break
    ins = []
    for i, ln in enumerate(lines):
        s = ln.strip()
        if not s or s.startswith((";", ".")) or s.endswith(":"):
            continue
        op, _, rest = s.partition(" ")
        rest = rest.split(";")[0]
        parts = [p.strip() for p in rest.split(",")]
        d, u = [], []
        if parts and parts[0] and not op.startswith(STORE_LIKE):
            d = regs(parts[0])
            for p in parts[1:]:
                u += regs(p)
            if op.startswith("v_mfma"):  # accumulator input may alias the output
                pass
        else:
            for p in parts:
                u += regs(p)
        ins.append((i, op, d, u))
    last = {}
    for k, (_, _, d, u) in enumerate(ins):
        for r in u + d:
            last[r] = k
    live, first_def, peak = set(), {}, []
    for k, (i, op, d, u) in enumerate(ins):
        for r in d:
            live.add(r)
        peak.append((len(live), i, op))
        for r in u + d:
            if last.get(r) == k:
                live.discard(r)
    top = sorted(peak, reverse=True)[:5]
    print("peak approx live regs:", top[0][0])
    for n, i, op in top:
        print(f"  {n:4d} at asm line {i}: {op}")
    step = max(1, len(peak) // int(window))
    for k in range(0, len(peak), step):
        n, i, op = peak[k]
        print(f"{i:6d} {n:4d} {'#' * (n // 4)} {op}")


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2], int(sys.argv[3]) if len(sys.argv) > 3 else 40)
