"""Where the batch-1 drop-in call's time goes (diagnostic; run on the GPU box).

    python tools/latency_breakdown.py [--dtype mixed] [--reps 50]

Times inference.run_unet end to end (median of --reps), then its stages one at a time: the
host-side cost of each call (perf_counter around the call, no sync) and the device time of the
preprocess and forward launches (HIP events on the launch stream), the device-to-host copy +
sync, and the host crops.  Prints one JSON line.
"""
import argparse
import json
import os
import sys
import tempfile
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tw-invoice-unet-ocr-llm_amd"))
sys.path.insert(0, REPO)

import numpy as np  # noqa: E402
import torch  # noqa: E402
from PIL import Image  # noqa: E402

from unet_mi355x import inference as inf  # noqa: E402
from unet_mi355x import synthetic as syn  # noqa: E402


def med(f, reps):
    t = []
    for _ in range(reps):
        t0 = time.perf_counter()
        f()
        t.append(time.perf_counter() - t0)
    return round(1e3 * float(np.median(t)), 4)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--dtype", default="mixed")
    ap.add_argument("--reps", type=int, default=50)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    inf.DEVICE = str(dev)
    page = syn.invoice_pages(7, 1, 400, 600, 1)[0, 0]
    pil = Image.fromarray((np.stack([page, page * 0.97, page * 0.94], -1) * 255 + 0.5).astype(np.uint8), "RGB")
    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in syn.make_state_dict(0, 3, 3, "pretrained").items()}
    out = {"dtype": a.dtype}
    with tempfile.TemporaryDirectory() as td:
        ck = os.path.join(td, "best_unet_model.pth")
        torch.save(sd, ck)
        for _ in range(3):
            inf.run_unet(pil, ck, compute_dtype=a.dtype)
        out["run_unet_ms"] = med(lambda: inf.run_unet(pil, ck, compute_dtype=a.dtype), a.reps)
        model = inf._cached_model(ck, a.dtype)
        st = inf._staging[str(dev)]
        stream = torch.cuda.current_stream(dev)
        out["cached_model_ms"] = med(lambda: inf._cached_model(ck, a.dtype), a.reps)
        out["native_handle_ms"] = med(lambda: model.native_handle(dev), a.reps)
        out["np_asarray_ms"] = med(lambda: np.asarray(pil), a.reps)
        arr = np.asarray(pil)
        out["upload_host_ms"] = med(lambda: st.upload(arr), a.reps)
        img = st.upload(arr)
        torch.cuda.synchronize()
        out["preprocess_host_ms"] = med(lambda: model.preprocess(img, 512, out=st.x[0]), a.reps)
        torch.cuda.synchronize()
        out["forward_boxes_host_ms"] = med(lambda: model.forward_boxes(st.x, masks="u8", out=(st.m, st.b)), a.reps)
        torch.cuda.synchronize()
        e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]

        def dev_times():
            e[0].record(stream)
            model.preprocess(img, 512, out=st.x[0])
            e[1].record(stream)
            model.forward_boxes(st.x, masks="u8", out=(st.m, st.b))
            e[2].record(stream)
            torch.cuda.synchronize()
            return e[0].elapsed_time(e[1]), e[1].elapsed_time(e[2])
        t = np.array([dev_times() for _ in range(a.reps)])
        out["preprocess_dev_ms"] = round(float(np.median(t[:, 0])), 4)
        out["forward_boxes_dev_ms"] = round(float(np.median(t[:, 1])), 4)

        def d2h():
            st.hm.copy_(st.m, non_blocking=True)
            st.hb.copy_(st.b, non_blocking=True)
            stream.synchronize()
        out["d2h_sync_ms"] = med(d2h, a.reps)
        out["mask_copy_ms"] = med(lambda: st.hm.numpy()[0].view(np.bool_).copy(), a.reps)
        boxes = st.hb.numpy()[0].copy()
        out["host_crops_ms"] = med(lambda: inf.boxes_to_crops(pil, boxes), a.reps)   # the host path (pixels read)
        rects, sums = st.hr.numpy().copy(), st.hs.numpy().copy()
        out["stats_crops_ms"] = med(lambda: [inf.crop_from_stats(pil, rects[i], sums[i], 3) for i in range(3)], a.reps)
        out["empty_sync_ms"] = med(lambda: stream.synchronize(), a.reps)
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
