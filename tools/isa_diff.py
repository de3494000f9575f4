"""Per-kernel ISA comparison of two `hipcc --cuda-device-only -S` outputs of csrc/unet_kernels.hip.

    python tools/isa_diff.py before.s after.s [--show KERNEL_SUBSTRING]

For every kernel symbol in both files: identical / differing (with the count of differing
instruction lines); kernels only in one file are listed.  Comments, labels' numbering and the
kernel descriptor (.amdhsa_*, kernarg sizes) are ignored: only the instruction stream counts.
"""
import difflib
import re
import sys


def kernels(path):
    out, cur, body = {}, None, []
    for line in open(path):
        m = re.match(r"^(_Z\w+):\s*(;.*)?$", line)
        if m:
            cur, body = m.group(1), []
            continue
        if cur is not None:
            if line.startswith(".Lfunc_end") or line.strip().startswith(".section"):
                out[cur] = body
                cur = None
                continue
            t = line.split(";")[0].strip()
            if not t or t.startswith(".") or t.endswith(":"):
                continue
            t = re.sub(r"\.LBB\d+_\d+", ".LBB", t)
            out.setdefault(cur, None)
            body.append(t)
    return {k: v for k, v in out.items() if v is not None}


def main():
    a, b = kernels(sys.argv[1]), kernels(sys.argv[2])
    show = sys.argv[sys.argv.index("--show") + 1] if "--show" in sys.argv else None
    same = diff = 0
    for k in sorted(set(a) & set(b)):
        if a[k] == b[k]:
            same += 1
            continue
        diff += 1
        d = [l for l in difflib.unified_diff(a[k], b[k], lineterm="", n=0) if l[:1] in "+-" and l[:3] not in ("+++", "---")]
        print(f"DIFF {len(d):5d} lines  {len(a[k])} -> {len(b[k])} instr  {k}")
        if show and show in k:
            print("\n".join(d[:200]))
    for k in sorted(set(a) - set(b)):
        print(f"ONLY-BEFORE {k}")
    for k in sorted(set(b) - set(a)):
        print(f"ONLY-AFTER  {k}")
    print(f"identical {same}, differing {diff}, removed {len(set(a) - set(b))}, added {len(set(b) - set(a))}")


if __name__ == "__main__":
    main()
