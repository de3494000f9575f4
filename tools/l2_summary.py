"""Per-launch L2 hit rate and L2->fabric read requests of the last forward of two rocprofv3 --pmc passes
(pass1: TCC_HIT_sum TCC_MISS_sum, pass2: TCC_EA0_RDREQ_sum TCC_EA0_RDREQ_DRAM_sum), each
`rocprofv3 --kernel-trace --pmc ... -d DIR/passN -o run -- python3 bench.py --steps 1 --warmup 0 ...`.
Usage: python tools/l2_summary.py DIR"""
import csv, collections, sys
labels = "down1.0 down1.3 down2.0 down2.3 down3.0 down3.3 down4.0 down4.3 bottleneck.0 bottleneck.3 up4 conv4.0 conv4.3 up3 conv3.0 conv3.3 up2 conv2.0 conv2.3+up1 conv1.0 conv1.3".split()
def load(path):
    d = collections.OrderedDict()
    for r in csv.DictReader(open(path)):
        if int(r["Grid_Size"]) < 10000: continue
        k = int(r["Dispatch_Id"]); d.setdefault(k, {"name": r["Kernel_Name"]})[r["Counter_Name"]] = float(r["Counter_Value"])
    return list(d.values())[-21:]
a = load(sys.argv[1] + "/pass1/run_counter_collection.csv")
b = load(sys.argv[1] + "/pass2/run_counter_collection.csv")
print("%-13s %7s %9s %9s %10s %10s" % ("launch", "L2hit%", "hit_M", "miss_M", "EA_rdreq_M", "dram_rdreq_M"))
for l, x, y in zip(labels, a, b):
    h, m = x["TCC_HIT_sum"], x["TCC_MISS_sum"]
    print("%-13s %7.1f %9.1f %9.1f %10.1f %10.1f" % (l, 100 * h / (h + m), h / 1e6, m / 1e6, y.get("TCC_EA0_RDREQ_sum", 0) / 1e6, y.get("TCC_EA0_RDREQ_DRAM_sum", 0) / 1e6))
