"""Build gate on the kernels' resource usage (hipcc -Rpass-analysis=kernel-resource-usage remarks,
written by the Makefile to csrc/build/unet_kernels.resources.txt).

Fails the build when a 16-bit kernel (the products' path: mangled template arguments DF16b / DF16_)
uses scratch or spills VGPRs: a register array indexed with a runtime value silently moves to
scratch and costs 5x (round 3: a runtime halo-chunk index in down1.3's fused first conv, 5.4 ->
26 ms).  Prints the table of every kernel.  Known and allowed, none on a default plan: the fp32
8-wave ring at TC = 8 and the 4-wave ring's pooled 128-row instantiation (2 spilled VGPRs).

    python tools/check_resources.py csrc/build/unet_kernels.resources.txt
"""
import re
import sys


def parse(path):
    kernels, cur = [], None
    for line in open(path, errors="replace"):
        m = re.search(r"remark: Function Name: (\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            kernels.append(cur)
            continue
        m = re.search(r"remark:\s+([A-Za-z ]+?)(?: \[[^\]]*\])?: (\S+) \[-Rpass", line)
        if m and cur is not None:
            cur[m.group(1).strip()] = m.group(2)
        elif "warning:" in line or "error:" in line:
            print(line.rstrip(), file=sys.stderr)
    return kernels


def main():
    ks = parse(sys.argv[1])
    bad = []
    for k in ks:
        scratch, spill = int(k.get("ScratchSize", 0)), int(k.get("VGPRs Spill", 0))
        gated = "DF16" in k["name"] and "conv3x3_ring_kernel" not in k["name"]
        if gated and (scratch or spill):
            bad.append(k)
        if scratch or spill or "ring8" in k["name"] or "convT" in k["name"]:
            print(f"{k.get('VGPRs', '?'):>4} VGPR {k.get('AGPRs', '?'):>3} AGPR  scratch {scratch:4}  spill {spill:3}  "
                  f"{k['name'][:110]}")
    if not ks:
        sys.exit("check_resources: no kernel-resource-usage remarks found")
    if bad:
        sys.exit(f"check_resources: {len(bad)} 16-bit kernel(s) use scratch or spill VGPRs: "
                 + ", ".join(k["name"] for k in bad))


if __name__ == "__main__":
    main()
