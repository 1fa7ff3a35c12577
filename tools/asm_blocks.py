"""Per-basic-block instruction mix of one render kernel in hipcc's device assembly
(`hipcc ... --cuda-device-only -S -o k.s rtx_hip.hip`): SALU / VALU / branch counts with the
loop nesting the compiler annotates, to find where the scalar work sits.
Usage: python tools/asm_blocks.py k.s [kernel-prefix]   (default: rtx_render_kernel<false, 0>)"""
import re
import sys


def main() -> None:
    lines = open(sys.argv[1]).read().split("\n")
    pref = sys.argv[2] if len(sys.argv) > 2 else "_Z17rtx_render_kernelILb0ELi0E"
    start = next(i for i, l in enumerate(lines) if l.startswith(pref) and ":" in l)
    end = next(i for i in range(start, len(lines)) if "s_endpgm" in lines[i])
    blocks, cur = [], None
    for l in lines[start:end + 1]:
        m = re.match(r"^(\.LBB\d+_\d+|; %bb\.\d+):?(.*)", l)
        if m:
            cur = {"name": m.group(1), "info": m.group(2).strip(" ;"), "s": 0, "v": 0, "b": 0, "first": []}
            blocks.append(cur)
            continue
        t = l.strip().split()
        if not t or cur is None or t[0].startswith((";", ".")):
            continue
        op = t[0]
        if op.startswith(("s_cbranch", "s_branch")):
            cur["b"] += 1
        elif op.startswith("s_") and not op.startswith(("s_waitcnt", "s_load", "s_nop", "s_endpgm")):
            cur["s"] += 1
        elif op.startswith("v_"):
            cur["v"] += 1
        if len(cur["first"]) < 3:
            cur["first"].append(op)
    for b in blocks:
        if b["s"] + b["v"]:
            d = re.search(r"Depth=(\d+)", b["info"])
            print(f"{b['name']:12s} d{d.group(1) if d else 0} s{b['s']:3d} v{b['v']:4d} b{b['b']}  "
                  f"{' '.join(b['first'])}")


if __name__ == "__main__":
    main()
