"""Where the batch-1 run_unet time goes beyond the forward (GPU box).

Times the drop-in run_unet (inference.py:50-129 restated in unet_mi355x/inference.py) on a
600x400 RGB photo at the fp32 default and the mixed plan: the end-to-end median, a cProfile of
the host side, and each stage of the call on its own (host wall time with a synchronisation
after the stage, and the device time of the stage between HIP events) -- the photo graph that
run_unet launches (round 5) and, for reference, its pieces as separate calls.
Usage: python tools/prof_run_unet.py [--calls 50]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import tempfile
import time

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tw-invoice-unet-ocr-llm_amd"))
from PIL import Image  # noqa: E402
from unet_mi355x import inference as inf, native  # noqa: E402
from unet_mi355x.model import UNet  # noqa: E402


def med(f, n):
    lat = []
    for _ in range(n):
        t0 = time.perf_counter()
        f()
        lat.append(time.perf_counter() - t0)
    return 1e3 * float(np.median(lat))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=50)
    args = ap.parse_args()
    dev = torch.device("cuda:0")
    inf.DEVICE = "cuda:0"
    # the bench's latency photo and weights (bench.py gpu_latency): a synthetic 600x400 invoice page and
    # the trained-like "pretrained" weights, so the fields' masks and crops are not empty
    from unet_mi355x import synthetic as syn
    sd = {k: torch.from_numpy(np.asarray(v)) for k, v in syn.make_state_dict(0, 3, 3, "pretrained").items()}
    page = syn.invoice_pages(7, 1, 400, 600, 1)[0, 0]
    pil = Image.fromarray((np.stack([page, page * 0.97, page * 0.94], -1) * 255 + 0.5).astype(np.uint8), "RGB")
    with tempfile.TemporaryDirectory() as td:
        ck = os.path.join(td, "best_unet_model.pth")
        torch.save(sd, ck)
        for dtype in ("fp32", "mixed"):
            for _ in range(5):
                inf.run_unet(pil, ck, compute_dtype=dtype)
            torch.cuda.synchronize()
            total = med(lambda: inf.run_unet(pil, ck, compute_dtype=dtype), args.calls)
            print(f"[{dtype}] run_unet median {total:.3f} ms over {args.calls} calls", flush=True)
            # the serving call over 16 photos (exact: chunks of the small-batch limit; loose: one forward)
            for exact in (True, False):
                batch = [pil] * 16
                inf.run_unet_batch(batch, ck, compute_dtype=dtype, exact=exact)
                tb = med(lambda: inf.run_unet_batch(batch, ck, compute_dtype=dtype, exact=exact), 7)
                print(f"[{dtype}] run_unet_batch x16 exact={exact}: {tb:.3f} ms = {tb / 16:.3f} ms per photo", flush=True)
            pr = cProfile.Profile()
            pr.enable()
            for _ in range(args.calls):
                inf.run_unet(pil, ck, compute_dtype=dtype)
            pr.disable()
            s = io.StringIO()
            pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(22)
            print(s.getvalue(), flush=True)

            # run_unet's RGB path step by step (the same calls), host time per section
            secs = {}
            for it in range(args.calls + 3):
                t = [time.perf_counter()]
                model_ = inf._cached_model(ck, dtype)
                t.append(time.perf_counter())
                st_ = inf._staging[str(inf.DEVICE)]
                with st_.lock, torch.no_grad():
                    stream_ = torch.cuda.current_stream(st_.device)
                    t.append(time.perf_counter())
                    img_, ch_ = st_.stage_photo(pil)
                    t.append(time.perf_counter())
                    blk_ = st_.mask_block()
                    g_ = st_.photo_graph(model_, img_, blk_)
                    g_.launch(stream_.cuda_stream)
                    t.append(time.perf_counter())
                    stream_.synchronize()
                    t.append(time.perf_counter())
                    m_ = st_.mask_blocks[blk_][1] if blk_ >= 0 else st_.hm.numpy()[0].view(np.bool_).copy()
                    rects_, sums_ = st_.hr.numpy().copy(), st_.hs.numpy().copy()
                    masks_ = {k: m_[i] for i, k in enumerate(inf.FIELDS)}
                    t.append(time.perf_counter())
                    crops_ = {k: inf.crop_from_stats(pil, rects_[i], sums_[i], ch_) for i, k in enumerate(inf.FIELDS)}
                    t.append(time.perf_counter())
                if it >= 3:
                    for j, name in enumerate(["cached_model", "lock+no_grad+stream", "stage_photo", "block+graph+launch",
                                              "synchronize", "masks (views)+rects", "crops"]):
                        secs.setdefault(name, []).append(t[j + 1] - t[j])
            # the masks out of the pinned buffer right after the graph's DMA wrote it (cold): numpy's
            # single-threaded copy against torch's parallel CPU copy into a fresh array
            cold = {"numpy": [], "torch": []}
            gc_ = st_.photo_graph(model_, img_, -1)   # the graph that DMAs into the shared pinned buffer
            for it in range(2 * args.calls + 6):
                gc_.launch(stream_.cuda_stream)
                stream_.synchronize()
                how = "numpy" if it % 2 == 0 else "torch"
                t0 = time.perf_counter()
                if how == "numpy":
                    mm = st_.hm.numpy()[0].view(np.bool_).copy()
                else:
                    mm = np.empty(st_.hm.shape[1:], dtype=np.bool_)
                    torch.from_numpy(mm.view(np.uint8)).copy_(st_.hm[0])
                cold[how].append(time.perf_counter() - t0)
                assert mm.shape == (3, 512, 512)
            print(f"[{dtype}] cold mask copy (median us): " +
                  ", ".join(f"{k} {1e6 * float(np.median(v[3:])):.1f}" for k, v in cold.items()), flush=True)
            print(f"[{dtype}] run_unet sections (median us): " +
                  ", ".join(f"{k} {1e6 * float(np.median(v)):.1f}" for k, v in secs.items()), flush=True)

            # the stages of run_unet, each followed by a synchronisation
            model = inf._cached_model(ck, dtype)
            st = inf._staging[str(inf.DEVICE)]
            stream = torch.cuda.current_stream(dev)
            arr = inf.photo_array(pil)
            img, _ = st.stage_photo(pil)
            graph = st.photo_graph(model, img)
            img = st.upload(arr)
            stages = {
                "cached_model": lambda: inf._cached_model(ck, dtype),
                "stage_photo": lambda: st.stage_photo(pil),   # run_unet's (RGB: RGBX export into pinned memory)
                "photo_array": lambda: inf.photo_array(pil),
                "stage_pinned": lambda: st.stage(arr),
                # the whole device part of the call as run_unet launches it: upload, resize, forward, boxes,
                # crop statistics and the four copies back, one graph
                "photo_graph": lambda: graph.launch(stream.cuda_stream),
                "upload": lambda: st.upload(arr),
                "preprocess": lambda: model.preprocess(img, inf.IMG_SIZE, out=st.x[0]),
                "forward_boxes": lambda: model.forward_boxes(st.x, masks="u8", out=(st.m, st.b)),
                "crop_stats": lambda: native.crop_stats(img, st.b[0], inf.IMG_SIZE, inf.IMG_SIZE, inf.CROP_PAD,
                                                        st.r, st.s, stream.cuda_stream),
                "d2h_4": lambda: (st.hr.copy_(st.r, non_blocking=True), st.hs.copy_(st.s, non_blocking=True),
                                  st.hm.copy_(st.m, non_blocking=True), st.hb.copy_(st.b, non_blocking=True)),
                "d2h_masks_only": lambda: st.hm.copy_(st.m, non_blocking=True),
                "mask_bool_copy": lambda: st.hm.numpy()[0].view(np.bool_).copy(),
                "crops": lambda: {k: inf.crop_from_stats(pil, st.hr.numpy()[i], st.hs.numpy()[i], 3)
                                  for i, k in enumerate(inf.FIELDS)},
                "sync_only": lambda: None,
            }
            for name, f in stages.items():
                def g():
                    f()
                    stream.synchronize()
                for _ in range(3):
                    g()
                host = med(g, args.calls)
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    f()
                e1.record()
                torch.cuda.synchronize()
                print(f"[{dtype}] {name:16s} host+sync {host:.4f} ms   device {e0.elapsed_time(e1) / 20:.4f} ms",
                      flush=True)
            # the crops with Pillow's block cache on (freed image blocks are kept for reuse instead of
            # returned to the OS: no page faults on the new crop's pixels)
            crops = {k: inf.crop_from_stats(pil, st.hr.numpy()[i], st.hs.numpy()[i], 3) for i, k in enumerate(inf.FIELDS)}
            print(f"[{dtype}] crop sizes " + ", ".join(f"{k}: {None if c is None else c.size}" for k, c in crops.items()))
            prev = Image.core.get_blocks_max()
            Image.core.set_blocks_max(8)
            f = stages["crops"]
            for _ in range(3):
                f()
            print(f"[{dtype}] crops with Pillow blocks_max 8: {med(f, args.calls):.4f} ms", flush=True)
            Image.core.set_blocks_max(prev)
            # the crops on worker threads (Pillow's crop copies rows with the GIL released)
            from concurrent.futures import ThreadPoolExecutor
            ex = ThreadPoolExecutor(2)
            rr, ss = st.hr.numpy(), st.hs.numpy()

            def pooled():
                fs = [ex.submit(inf.crop_from_stats, pil, rr[i], ss[i], 3) for i in range(1, 3)]
                c0 = inf.crop_from_stats(pil, rr[0], ss[0], 3)
                return [c0] + [x.result() for x in fs]
            for _ in range(3):
                pooled()
            print(f"[{dtype}] crops on 2 pool threads + caller: {med(pooled, args.calls):.4f} ms", flush=True)
            ex.shutdown()
            with torch.no_grad():
                x = st.x
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(20):
                    model.forward_boxes(x, masks="u8", out=(st.m, st.b))
                e1.record()
                torch.cuda.synchronize()
                t = med(lambda: model.forward_boxes(x, masks="u8", out=(st.m, st.b)), args.calls)
                print(f"[{dtype}] forward_boxes host enqueue {t:.4f} ms (no sync)", flush=True)


if __name__ == "__main__":
    main()
