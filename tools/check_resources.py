"""Build gate on the kernels' resource usage (hipcc -Rpass-analysis=kernel-resource-usage remarks,
written by the Makefile to csrc/build/unet_kernels.resources.txt).

Fails the build when any kernel of the product library uses scratch or spills VGPRs: a register
array indexed with a runtime value silently moves to scratch and costs 5x (round 3: a runtime
halo-chunk index in down1.3's fused first conv, 5.4 -> 26 ms).  No allow-list: configurations whose
instantiation would spill (the fp32 128-row 8-wave ring, the pooled 128-row 4-wave ring) are not built
(unet_kernels.hip launch_3x3; unet_capi.cpp maps them to the 64-row tiles of the same family).
Prints the table of every ring / ConvTranspose kernel and of any that spills.

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
        if scratch or spill:
            bad.append(k)
        if scratch or spill or "ring8" in k["name"] or "convT" in k["name"]:
            print(f"{k.get('VGPRs', '?'):>4} VGPR {k.get('AGPRs', '?'):>3} AGPR  scratch {scratch:4}  spill {spill:3}  "
                  f"{k['name'][:110]}")
    if not ks:
        sys.exit("check_resources: no kernel-resource-usage remarks found")
    if bad:
        sys.exit(f"check_resources: {len(bad)} kernel(s) use scratch or spill VGPRs: "
                 + ", ".join(k["name"] for k in bad))


if __name__ == "__main__":
    main()
