"""Explain the read traffic (2 x FETCH_SIZE) of the 128-row 3x3 ring launches.

Model: every launch reads its input once, and every XCD re-streams ALL of the layer's weights
once per round of pixel tiles -- one block per CU, the n_ct row tiles of a walker on one XCD
(consecutive block ids), so the 32 blocks of an XCD cover every row tile and, per round, touch
the whole weight tensor, which exceeds the XCD's 4 MiB L2 on the deep layers.
  rounds = ceil(pixel tiles / walkers), walkers = 256 / n_ct, n_ct = Cout / 128, tiles 16 x 32.
Usage: python tools/traffic_model.py profiles/pmc_r2o_mixed_bs256_summary.txt
"""
import math
import sys

N = 256  # images per step (bench config)
# (launch label, Cin, Cout, H = W at this level, bytes per element)
LAYERS = [("down2.0", 64, 128, 256, 2), ("down2.3", 128, 128, 256, 2), ("down3.0", 128, 256, 128, 2),
          ("down3.3", 256, 256, 128, 2), ("down4.0", 256, 512, 64, 2), ("down4.3", 512, 512, 64, 2),
          ("bottleneck.0", 512, 1024, 32, 2), ("bottleneck.3", 1024, 1024, 32, 2), ("conv4.0", 1024, 512, 64, 2),
          ("conv4.3", 512, 512, 64, 2), ("conv3.0", 512, 256, 128, 2), ("conv3.3", 256, 256, 128, 2),
          ("conv2.0", 256, 128, 256, 2)]


def main(path):
    meas = {}
    for line in open(path):
        p = line.split()
        if len(p) == 7 and p[0] != "launch" and p[0][0].isalpha():
            meas[p[0]] = float(p[1])
    print("%-13s %5s %6s %8s %9s %8s %8s %6s" % ("layer", "n_ct", "rounds", "input_GB", "weights_GB", "model", "read_GB", "ratio"))
    for name, cin, cout, hw, b in LAYERS:
        n_ct = cout // 128
        walkers = 256 // n_ct
        rounds = math.ceil(N * (hw // 16) * (hw // 32) / walkers)
        inp = N * hw * hw * cin * b / 1e9
        w = cin * cout * 9 * b / 1e9 * rounds * 8
        m = meas.get(name, float("nan"))
        print("%-13s %5d %6d %8.2f %9.2f %8.2f %8.2f %6.2f" % (name, n_ct, rounds, inp, w, inp + w, m, m / (inp + w)))


if __name__ == "__main__":
    main(sys.argv[1] if len(sys.argv) > 1 else "profiles/pmc_r2o_mixed_bs256_summary.txt")
