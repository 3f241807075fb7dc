"""Throughput of the extraction hot path on MI355X.

metric : extracted frames/sec, 512x424 depth video, batch = 32 (BASELINE.json)
step   : one pass of the hot path over one batch of 32 synthetic raw int16
         512x424 frames already resident in HBM:
         prep_raw_frames (bg subtract, ROI, clamp, NS inpaint) -> scale (fused)
         -> R50-FPN Mask/Keypoint R-CNN forward (fp16 MFMA, SCORE_THRESH_TEST=0
         so every frame carries exactly 4 detections) -> mask-IoU NMS +
         instance-0 selection -> clean_frames (median3 + 3x open ellipse9)
         -> moments -> angle -> crop_and_rotate (depth + mask).
value  : frames processed by all ranks / max-over-ranks wall time.
scaling: weak (every rank processes its own 32-frame batches; frames shard
         with no data-path collective; N>1 gathers each step's 80x80 crops to
         rank 0 over RCCL, the reference's result hand-off to the writer).

Launch: python bench.py [--gpus N --steps K --warmup W]
        (N>1 via torch.distributed.run, one process per GPU)
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)
# One HIP hardware queue per stream of the overlapped pipeline (default, front,
# two model forwards, tail): with HIP's default of 4 the tail shares a queue
# with a model stream, and its wait for one forward blocks the next forward
# queued behind it (measured +2.7 % with 8).  Read at HIP initialisation.
os.environ["GPU_MAX_HW_QUEUES"] = "8"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--dtype", default="fp16", choices=["fp16", "fp32"])
    ap.add_argument("--depth", type=int, default=50, choices=[50, 101])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--issue-stream", type=int, default=1, help="issue the pipeline from a pool stream (1) or the NULL stream (0)")
    ap.add_argument("--cpu-sample-frames", type=int, default=2)
    ap.add_argument("--dump-convs", default=None, help="write per-launch conv timings (JSON) to this path")
    ap.add_argument("--no-overlap", action="store_true",
                    help="run batches back to back on one stream instead of the multi-stream pipeline")
    ap.add_argument("--dma128", type=int, default=None, help="conv kernel policy knob (mdx_conv_set_dma128)")
    ap.add_argument("--prio256", type=int, default=None, help="conv knob (mdx_conv_set_mfma_prio256)")
    ap.add_argument("--stream1x1", type=int, default=None, help="conv knob (mdx_conv_set_stream1x1)")
    ap.add_argument("--stream-min-m", type=int, default=65536, help="conv knob (mdx_conv_set_stream1x1 min_m)")
    ap.add_argument("--dma-after", type=int, default=None, help="conv knob (mdx_conv_set_dma_after)")
    ap.add_argument("--roi-mode", type=int, default=None, help="ROIAlign kernel (mdx_roi_align_set_mode)")
    ap.add_argument("--model-streams", type=int, default=2,
                    help="forwards of consecutive batches in flight at once (one HIP stream each)")
    return ap.parse_args()


KERNEL_SYMBOLS = {  # MDX_CONV_KERNEL_* -> rocprofv3 symbol (fp16 in / fp16 out)
    0: "_ZN3mdx6k_convIDF16_DF16_Li128EEEvNS_8ConvArgsE",
    1: "_ZN3mdx6k_convIDF16_DF16_Li64EEEvNS_8ConvArgsE",
    2: "_ZN3mdx7k_convgIDF16_Li8ELb0ELb0ELb0EEEvNS_8ConvArgsE",
    3: "_ZN3mdx7k_convgIDF16_Li4ELb1ELb0ELb0EEEvNS_8ConvArgsE",
    4: "k_conv1x1_stream<KC> (three instances by K)",
    5: "k_conv1x1_head<KC> (three instances by K)",
}
KERNEL_NAMES = {0: "k_conv<128> register-staged implicit GEMM", 1: "k_conv<64> register-staged implicit GEMM",
                2: "k_convg<8> 256x256 LDS-DMA implicit GEMM", 3: "k_convg<4> 128x128 LDS-DMA implicit GEMM",
                4: "k_conv1x1_stream streaming 1x1 GEMM", 5: "k_conv1x1_head narrow-output streaming 1x1"}


def conv_roofline(extractor, raw, steps=3, dump=None):
    """Time every conv launch of a step with HIP events on the launch stream
    and tag it with the kernel the library chose (mdx_conv2d_last_plan).
    Returns {kernel id: [algorithmic FLOP, seconds, launches]} per step plus
    the totals over all conv launches."""
    import ctypes
    import torch
    from moseq2_detectron_extract_amd._lib import call
    from moseq2_detectron_extract_amd.model import runtime as RT
    rec = []
    orig = RT.MaskRCNN.conv
    kid, ksp = ctypes.c_int(), ctypes.c_int()

    def timed(self, x, N, H, W, c, relu, out=None, residual=None, out_f32=False, out_mode=0):
        s = torch.cuda.current_stream()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(s)
        r = orig(self, x, N, H, W, c, relu, out, residual, out_f32, out_mode)
        e1.record(s)
        call("mdx_conv2d_last_plan", ctypes.byref(kid), ctypes.byref(ksp))
        OH, OW = r[1], r[2]
        kalg = c.kalg or c.k * c.k * c.cin
        key = kid.value if not out_f32 else kid.value + 10  # fp32-output instances are other symbols
        rec.append((e0, e1, 2.0 * N * OH * OW * c.cout * kalg, key, ksp.value,
                    (N * OH * OW, c.cout, c.k * c.k * c.cin, c.k, c.stride, out_mode, residual is not None)))
        return r

    RT.MaskRCNN.conv = timed
    try:
        for _ in range(steps):
            extractor.step_device(raw)
        torch.cuda.synchronize()
    finally:
        RT.MaskRCNN.conv = orig
    per = {}
    for e0, e1, f, key, ks, _ in rec:
        d = per.setdefault(key, [0.0, 0.0, 0, 0])
        d[0] += f / steps
        d[1] += e0.elapsed_time(e1) * 1e-3 / steps
        d[2] += 1.0 / steps
        d[3] = max(d[3], ks)
    if dump:
        n = len(rec) // steps
        rows = [{"M": sh[0], "N": sh[1], "K": sh[2], "k": sh[3], "stride": sh[4], "mode": sh[5], "res": sh[6],
                 "kernel": key, "ksplit": ks, "us": e0.elapsed_time(e1) * 1e3,
                 "tflops": f / (e0.elapsed_time(e1) * 1e-3) / 1e12}
                for e0, e1, f, key, ks, sh in rec[-n:]]
        with open(dump, "w") as fh:
            json.dump(rows, fh, indent=0)
    return per


def roofline_line(per, dtype):
    """Roofline object for the dominant conv kernel (most time per step)."""
    peak = 2500.0 if dtype == "fp16" else 157.3
    key = max(per, key=lambda k: per[k][1])
    fl, sec, n, ks = per[key]
    ach = fl / sec / 1e12
    traffic = None
    sym = KERNEL_SYMBOLS.get(key)
    pmc = os.path.join(ROOT, "profiles", "r01_pmc_kernels.json")
    if sym and os.path.exists(pmc):
        try:
            with open(pmc) as fh:
                traffic = json.load(fh)["kernels"].get(sym, {}).get("hbm_bytes_per_launch")
        except Exception:
            traffic = None
    tot_f = sum(v[0] for v in per.values())
    tot_s = sum(v[1] for v in per.values())
    return {"bound": "mfma", "achieved": round(ach, 2), "peak": peak, "unit": "TFLOP/s",
            "frac": round(ach / peak, 4), "traffic": traffic,
            "kernel": f"{KERNEL_NAMES.get(key, key)} ({sym}): {n:.0f} launches/step, "
                      f"{fl / n / 1e9:.1f} GFLOP and {sec / n * 1e6:.1f} us per launch (HIP events on the launch "
                      f"stream; traffic = PMC HBM bytes per launch)",
            "all_conv": {"launches": round(sum(v[2] for v in per.values())), "tflop_per_step": round(tot_f / 1e12, 3),
                         "ms_per_step": round(tot_s * 1e3, 3), "achieved": round(tot_f / tot_s / 1e12, 1)}}


def cpu_baseline(nframes: int, dtype_cfg):
    """Oracle (CPU restatement) timed on the host cores: prep+inpaint (C),
    PyTorch-CPU fp32 model forward, clean/moments/crop (C)."""
    import numpy as np
    import torch
    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd import synth
    from moseq2_detectron_extract_amd.model import synthetic_state_dict
    from oracle import frameops as O
    from oracle import model_ref as R
    cores = len(os.sched_getaffinity(0))
    # the GPU box exposes the whole machine's cores but grants this job a share
    # (OMP_NUM_THREADS); oversubscribing 256 threads is far slower
    cores = min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))
    torch.set_num_threads(cores)
    s = synth.SyntheticSession(nframes, seed=123)
    raw = s.frames(0, nframes)
    sd = synthetic_state_dict(dtype_cfg, 0)
    t0 = time.perf_counter()
    prepped, _ = O.prep_raw_frames(raw, s.bground_im, s.roi, 0, 100)
    scaled = O.scale_raw_frames(prepped, 0, 100)
    res, _ = R.forward(sd, dtype_cfg, scaled[..., None], keep_intermediates=False)
    d2 = np.stack([r["pred_masks"][0].numpy().astype(np.uint8) if len(r["pred_masks"]) else
                   np.zeros(prepped.shape[1:], np.uint8) for r in res])
    cl = O.clean_frames(prepped, iters_tail=3)
    f = O.get_frame_features(cl, 3, mask=d2)
    ang = np.mod(-np.rad2deg(f["orientation"]), 360)
    O.crop_and_rotate_frames(prepped, f["centroid"], ang)
    O.crop_and_rotate_frames(d2, f["centroid"], ang)
    dt = time.perf_counter() - t0
    return {"value": nframes / dt, "unit": "frames/s", "cores": cores, "kind": "port",
            "sample": f"{nframes} synthetic 512x424 frames through the CPU oracle (C frame ops + PyTorch-CPU fp32 "
                      f"R50-FPN Mask/Keypoint R-CNN, SCORE_THRESH_TEST=0), {dt:.1f} s"}


def main():
    args = parse()
    import numpy as np
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)

    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd import synth
    from moseq2_detectron_extract_amd.model import ModelConfig, Predictor
    from moseq2_detectron_extract_amd.model.runtime import flops_per_image
    from moseq2_detectron_extract_amd.pipeline import ExtractConfig, GPUExtractor, OverlappedExtractor

    if args.dma128 is not None:
        from moseq2_detectron_extract_amd._lib import call
        call("mdx_conv_set_dma128", args.dma128, 1536)
    if args.stream1x1 is not None:
        from moseq2_detectron_extract_amd._lib import call
        call("mdx_conv_set_stream1x1", args.stream1x1, args.stream_min_m)
    if args.dma_after is not None:
        from moseq2_detectron_extract_amd._lib import call
        call("mdx_conv_set_dma_after", args.dma_after)
    if args.roi_mode is not None:
        from moseq2_detectron_extract_amd._lib import call
        call("mdx_roi_align_set_mode", args.roi_mode)
    if args.prio256 is not None:
        from moseq2_detectron_extract_amd._lib import call
        call("mdx_conv_set_mfma_prio256", args.prio256)
    B = args.batch
    cfg = ModelConfig(depth=args.depth, score_thresh_test=0.0)
    pred = Predictor.from_config(cfg, dtype=args.dtype, seed=0)
    sess = synth.SyntheticSession(2 * B, seed=1000 + rank)
    raw_all = torch.from_numpy(sess.frames(0, 2 * B)).cuda()
    ex = GPUExtractor(sess.bground_im, sess.roi, pred, ExtractConfig(batch_size=B))

    gather_bufs = None
    if world > 1:
        gather_bufs = [torch.empty((B, 2, 80, 80), dtype=torch.uint8, device="cuda") for _ in range(world)]

    pipe = None if args.no_overlap else OverlappedExtractor(ex, args.model_streams)

    gstream = torch.cuda.Stream() if world > 1 else None

    def deliver(r):
        if r is not None and world > 1:
            # on a side stream, so the hand-off never orders the caller's
            # stream (and the pipeline's next fronts) behind this batch
            with torch.cuda.stream(gstream):
                if "ready" in r:
                    gstream.wait_event(r["ready"])
                payload = torch.stack([r["depth_frames"], r["mask_frames"]], 1).contiguous()
                dist.gather(payload, gather_bufs if rank == 0 else None, dst=0)

    # the loop issues from a pool stream, not HIP's legacy NULL stream: an
    # event recorded on the NULL stream also waits for all earlier work of
    # every blocking stream, which would order each front behind the
    # previous forward
    issue_stream = torch.cuda.Stream() if args.issue_stream else torch.cuda.current_stream()

    def run(nsteps, offset):
        with torch.cuda.stream(issue_stream):
            run_(nsteps, offset)

    def run_(nsteps, offset):
        # nsteps batches through the path; with the pipeline the last batch is
        # flushed inside, so exactly nsteps batches complete
        for i in range(nsteps):
            raw = raw_all[((offset + i) % 2) * B:((offset + i) % 2) * B + B]
            deliver(ex.step_device(raw) if pipe is None else pipe.submit(raw))
        if pipe is not None:
            for r in pipe.flush():
                deliver(r)

    run(args.warmup, 0)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(args.steps, args.warmup)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    if world > 1:
        t = torch.tensor([dt], dtype=torch.float64, device="cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    frames = world * args.steps * B
    value = frames / dt

    roof = None
    if not args.no_roofline:
        per = conv_roofline(ex, raw_all[:B], dump=args.dump_convs)
        roof = roofline_line(per, args.dtype)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(args.cpu_sample_frames, ModelConfig(depth=args.depth, score_thresh_test=0.0))
        except Exception as e:  # the baseline must never sink the bench line
            cpu = {"value": None, "error": repr(e)[:200]}

    if rank == 0:
        line = {
            "metric": f"extracted frames/sec, 512x424 depth video batch={B}",
            "value": round(value, 2), "unit": "frames/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(dt / args.steps * 1e3, 3), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": args.dtype, "data": "synthetic",
            "config": {"workload": f"full extract hot path (prep+inpaint, scale, R{args.depth}-FPN Mask/Keypoint "
                                   f"R-CNN {args.dtype}, mask NMS, clean, moments, crop), 512x424 int16 frames",
                       "global_batch": B * world, "per_gpu_batch": B, "frame": [424, 512],
                       "model_gflop_per_frame": round(flops_per_image(cfg) / 1e9, 2),
                       "parallelism": f"frame-sharded x{world}",
                       "streams": "1" if args.no_overlap else f"{2 + args.model_streams} (prep/inpaint/clean of the "
                                  f"newest batch, {args.model_streams} model forwards + mask selection of the next "
                                  f"batches, moments/crop of the oldest)"},
            "roofline": roof, "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
