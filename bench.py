"""Throughput of the extraction hot path on MI355X.

metric : extracted frames/sec, 512x424 depth video, batch = 32 (BASELINE.json)
step   : one pass of the hot path over one batch of 32 synthetic raw int16
         512x424 frames that start in pinned HOST memory (the frame source's
         buffers): H2D copy (own stream, inside the timed region) ->
         prep_raw_frames (bg subtract, ROI, clamp, NS inpaint) -> scale (fused)
         -> R50-FPN Mask/Keypoint R-CNN forward (fp32 = the reference's
         precision; SCORE_THRESH_TEST=0 so every frame carries exactly 4
         detections) -> mask-IoU NMS + instance-0 selection -> clean_frames
         (median3 + 3x open ellipse9) -> moments -> angle -> crop_and_rotate
         (depth + mask).
loop   : the staggered five-stream pipeline (pipeline.OverlappedExtractor):
         H2D, prep/inpaint/clean of batch i+3, the forwards of batches i+1 and
         i+2 on two HIP streams, moments/crop of batch i, all concurrent;
         --chunked runs chunks of --chunk-batches (8) batches instead (the
         chunk's stages one after another, its forwards alternating over two
         streams: GPUExtractor.step_device), --no-overlap one batch at a time.
value  : frames processed by all ranks / max-over-ranks wall time.
scaling: weak (every rank processes its own 32-frame batches; frames shard
         with no data-path collective; N>1 gathers each step's 80x80 crops to
         rank 0 over RCCL, the reference's result hand-off to the writer).
secondary.fp16: the same loop with the fp16 MFMA forward (BASELINE config 5's
         precision), reported beside the fp32 headline, never as `value`.
secondary.fp32_bf16x6: the same loop with the fp32 layers as exact bf16
         plane products (mdx_policy.fp32_split = 6).
secondary.extract_loop: BASELINE config 3 -- extract.extract_session over a
         10k-frame synthetic session written as depth.dat (chunks of 1000,
         tracking on, fp32): frame source, device path, instance selection,
         the native Kalman / flip angle step, scalars, keypoint tables, crops
         and the result writers (results + keypoints TSV), frames / wall time.
roofline: the MFMA kernel with the most GPU time per serial step (HIP events
         around every conv launch; a Winograd layer's batched GEMM counts
         under the kernel it runs on, at its executed FLOPs), the other top
         kernels beside it, and frame_ops: the frame kernels' algorithmic HBM
         bytes / their HIP-event time vs 8 TB/s (+ PMC bytes from profiles/).

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
# HIP hardware queues: at least 12 (HIP's default is 4), set before the runtime
# initialises, so that the loop's streams -- H2D, front, eight model forwards,
# tail, the gather -- each get a queue of their own: with 4 queues a third
# model stream shared a queue with another stage and lost 2 %, with 8 it gained
# 2.5 % over two streams (1348 -> 1382 fps, profiles/r03_experiments.json), a
# fourth 0.7-1.0 % over three (profiles/r04_experiments.json), and at 12 queues
# eight forwards 2.3 % over four (1491 -> 1525-1528; 12 or 16 forwards no more,
# profiles/r06_model_streams/).
# Recorded in the line.  (The illegal-address faults once seen with 8 queues
# and three model streams were the inpaint set-up race, fixed: DESIGN.md §3.)
if int(os.environ.get("GPU_MAX_HW_QUEUES", "4")) < 12:
    os.environ["GPU_MAX_HW_QUEUES"] = "12"


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--batch", type=int, default=32)
    ap.add_argument("--dtype", default="fp32", choices=["fp16", "fp32", "mixed"],
                    help="mixed: fp32 backbone / FPN / RPN / box head, fp16 mask + keypoint heads (config 5 as stated)")
    ap.add_argument("--depth", type=int, default=50, choices=[50, 101])
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--no-roofline", action="store_true")
    ap.add_argument("--no-secondary", action="store_true", help="skip the fp16 secondary measurement")
    ap.add_argument("--no-x6", action="store_true",
                    help="skip the secondary fp32 loop on the split-plane kernels (mdx_policy.fp32_split = 6)")
    ap.add_argument("--no-h2d", action="store_true", help="raw batches already resident in HBM (no H2D in the loop)")
    ap.add_argument("--cpu-sample-frames", type=int, default=64)
    ap.add_argument("--no-extract-loop", action="store_true", help="skip the config-3 extract-loop secondary")
    ap.add_argument("--no-config5", action="store_true",
                    help="skip the config-5 secondary (R101-FPN B=64, fp16 mask + keypoint heads)")
    ap.add_argument("--extract-frames", type=int, default=10000)
    ap.add_argument("--extract-chunk", type=int, default=1000)
    ap.add_argument("--extract-per-chunk", action="store_true",
                    help="extract loop: drain the stream pipeline at every chunk (round-4 schedule, for A/B runs)")
    ap.add_argument("--dump-convs", default=None, help="write per-launch conv timings (JSON) to this path")
    ap.add_argument("--no-overlap", action="store_true",
                    help="run batches back to back on one stream (one forward at a time)")
    ap.add_argument("--pipeline", action="store_true",
                    help="software pipeline over streams (pipeline.OverlappedExtractor: front / forwards / tail of "
                         "consecutive batches concurrently) -- the default; kept for older command lines")
    ap.add_argument("--chunked", action="store_true",
                    help="the chunked loop (GPUExtractor.step_device over --chunk-batches batches) instead of the "
                         "pipeline")
    ap.add_argument("--roi-mode", type=int, default=None, help="ROIAlign kernel (mdx_policy.roi_mode)")
    ap.add_argument("--dma-f32", type=int, default=None, help="fp32 LDS-DMA conv policy (mdx_policy.dma_f32)")
    ap.add_argument("--winograd", type=int, default=None, help="fp32 3x3 Winograd policy (mdx_policy.winograd)")
    ap.add_argument("--winograd-min-cin", type=int, default=None, help="mdx_policy.winograd_min_cin")
    ap.add_argument("--set", action="append", default=[], metavar="FIELD=INT",
                    help="set a field of the kernel-selection policy (include/mdx.h mdx_policy) before the model "
                         "handles are created, e.g. --set rpn_sliced=0 (repeatable)")
    ap.add_argument("--model-streams", type=int, default=8,
                    help="forwards in flight at once (one HIP stream each)")
    ap.add_argument("--chunk-batches", type=int, default=8,
                    help="batches per chunk in the default loop (the chunk's forwards alternate over the streams)")
    args = ap.parse_args()
    args.pipeline = not args.chunked and not args.no_overlap
    return args


# MDX_CONV_KERNEL_* (+10: fp32-output instance of an fp16 model) -> rocprofv3 symbol, per dtype


def _kconv(ti: str, to: str, bn: int, dual: bool, pw: bool):
    """Mangled and demangled name of k_conv<TI, TO, BN, DUAL, PW>."""
    m = {"f32": ("f", "float"), "f16": ("DF16_", "_Float16")}
    b = lambda v: ("1", "true") if v else ("0", "false")  # noqa: E731
    mangled = f"_ZN3mdx6k_convI{m[ti][0]}{m[to][0]}Li{bn}ELb{b(dual)[0]}ELb{b(pw)[0]}EEEvNS_8ConvArgsE"
    return mangled, f"void mdx::k_conv<{m[ti][1]}, {m[to][1]}, {bn}, {b(dual)[1]}, {b(pw)[1]}>(mdx::ConvArgs)"


# kernel id -> (BN, DUAL, PW) of the k_conv instance (ids +10: fp16 in, fp32 out)
_KCONV_IDS = {0: (128, False, False), 1: (64, False, False), 14: (128, False, True), 15: (64, False, True),
              16: (128, True, True), 17: (64, True, True)}
KERNEL_SYMBOLS = {"fp16": {2: "_ZN3mdx7k_convgIDF16_DF16_Li8ELb0EEEvNS_8ConvArgsE",
                           3: "_ZN3mdx7k_convgIDF16_DF16_Li4ELb1EEEvNS_8ConvArgsE",
                           4: "k_conv1x1_stream<KC> (three instances by K)",
                           5: "k_conv1x1_head<KC> (three instances by K)"},
                  "fp32": {2: "_ZN3mdx7k_convgIffLi8ELb0EEEvNS_8ConvArgsE"}}
# rocprofv3 reports some kernels demangled
KERNEL_DEMANGLED = {
    "_ZN3mdx7k_convgIDF16_DF16_Li8ELb0EEEvNS_8ConvArgsE":
        "void mdx::k_convg<_Float16, _Float16, 8, false>(mdx::ConvArgs)",
    "_ZN3mdx7k_convgIffLi8ELb0EEEvNS_8ConvArgsE":
        "void mdx::k_convg<float, float, 8, false>(mdx::ConvArgs)",
}
for _k, _bn, _dual in ((18, 128, 0), (19, 64, 0), (20, 128, 1), (21, 64, 1)):  # k_conv_sb<T, T, BN, DUAL>
    for _dt, _mt, _dm in (("fp32", "ff", "float, float"), ("fp16", "DF16_DF16_", "_Float16, _Float16")):
        _m = f"_ZN3mdx9k_conv_sbI{_mt}Li{_bn}ELb{_dual}EEEvNS_8ConvArgsE"
        KERNEL_SYMBOLS[_dt][_k] = _m
        KERNEL_DEMANGLED[_m] = f"void mdx::k_conv_sb<{_dm}, {_bn}, {'true' if _dual else 'false'}>(mdx::ConvArgs)"
for _k, _bn in ((22, 128), (23, 64)):  # k_conv_sbg<T, T, BN>: single stage, general layers
    for _dt, _mt, _dm in (("fp32", "ff", "float, float"), ("fp16", "DF16_DF16_", "_Float16, _Float16")):
        _m = f"_ZN3mdx10k_conv_sbgI{_mt}Li{_bn}EEEvNS_8ConvArgsE"
        KERNEL_SYMBOLS[_dt][_k] = _m
        KERNEL_DEMANGLED[_m] = f"void mdx::k_conv_sbg<{_dm}, {_bn}>(mdx::ConvArgs)"
for _k, (_bn, _dual, _pw) in _KCONV_IDS.items():
    for _dt, _t in (("fp32", "f32"), ("fp16", "f16")):
        _m, _d = _kconv(_t, _t, _bn, _dual, _pw)
        KERNEL_SYMBOLS[_dt][_k] = _m
        KERNEL_DEMANGLED[_m] = _d
    if not _dual:
        _m, _d = _kconv("f16", "f32", _bn, False, _pw)
        KERNEL_SYMBOLS["fp16"][_k + 10] = _m
        KERNEL_DEMANGLED[_m] = _d
KERNEL_NAMES = {0: "k_conv<128> register-staged implicit GEMM", 1: "k_conv<64> register-staged implicit GEMM",
                2: "k_convg<8> 256x256 LDS-DMA implicit GEMM", 3: "k_convg<4> 128x128 LDS-DMA implicit GEMM",
                4: "k_conv1x1_stream streaming 1x1 GEMM", 5: "k_conv1x1_head narrow-output streaming 1x1",
                7: "k_conv_x3<128> fp32 as bf16 plane products", 8: "k_conv_x3<64> fp32 as bf16 plane products",
                9: "k_gemm_x6 256x256 LDS-DMA GEMM over bf16 planes (fp32 split, two plane products per MFMA)",
                10: "k_conv<128> fp32-output instance", 11: "k_conv<64> fp32-output instance",
                12: "k_wino_in Winograd input transform", 13: "k_wino_out Winograd output transform",
                14: "k_conv<128, PW> register-staged implicit GEMM, pointwise addressing",
                15: "k_conv<64, PW> register-staged implicit GEMM, pointwise addressing",
                16: "k_conv<128, DUAL> conv3 + projection shortcut GEMM",
                17: "k_conv<64, DUAL> conv3 + projection shortcut GEMM",
                18: "k_conv_sb<128> register-staged implicit GEMM, pointwise, single LDS stage (3 WG/CU)",
                19: "k_conv_sb<64> register-staged implicit GEMM, pointwise, single LDS stage (4 WG/CU)",
                20: "k_conv_sb<128, DUAL> conv3 + projection shortcut GEMM, single LDS stage",
                21: "k_conv_sb<64, DUAL> conv3 + projection shortcut GEMM, single LDS stage",
                22: "k_conv_sbg<128> register-staged implicit GEMM, single LDS stage",
                23: "k_conv_sbg<64> register-staged implicit GEMM, single LDS stage",
                24: "k_conv<128, PW> fp32-output instance", 25: "k_conv<64, PW> fp32-output instance",
                26: "k_conv16_pp 256x256 fp16 ping-pong implicit GEMM (two wave groups one barrier apart)"}
KERNEL_SYMBOLS["fp16"][26] = "_ZN3mdx11k_conv16_ppIDF16_EEvNS_8ConvArgsE"
KERNEL_DEMANGLED["_ZN3mdx11k_conv16_ppIDF16_EEvNS_8ConvArgsE"] = "void mdx::k_conv16_pp<_Float16>(mdx::ConvArgs)"
KERNEL_DEMANGLED["_ZN3mdx11k_conv16_ppIfEEvNS_8ConvArgsE"] = "void mdx::k_conv16_pp<float>(mdx::ConvArgs)"
# the transforms: one instance per Winograd tile size the default policy runs
# (F(6,3) on the large maps, F(4,3) on the rest)
KERNEL_SYMBOLS["fp32"].update({12: tuple(f"_ZN3mdx9k_wino_inILi{m}EEEvPKfiiiiiiPf" for m in (4, 6)),
                               13: tuple(f"_ZN3mdx10k_wino_outILi{m}EEEvPKfiiiiiiS2_iPf" for m in (4, 6))})
for _m in (4, 6):
    KERNEL_DEMANGLED[f"_ZN3mdx9k_wino_inILi{_m}EEEvPKfiiiiiiPf"] = \
        f"void mdx::k_wino_in<{_m}>(float const*, int, int, int, int, int, int, float*)"
    KERNEL_DEMANGLED[f"_ZN3mdx10k_wino_outILi{_m}EEEvPKfiiiiiiS2_iPf"] = \
        f"void mdx::k_wino_out<{_m}>(float const*, int, int, int, int, int, int, float const*, int, float*)"
TRANSFORMS = (12, 13)  # records whose "flop" field holds algorithmic HBM bytes
PEAK = {"fp16": 2500.0, "fp32": 157.3}  # dense TFLOP/s, MI355X_MICROARCH.md
HBM_PEAK = 8000.0  # GB/s, MI355X_MICROARCH.md
PMC_FILE = {"fp16": "r06_pmc_kernels_fp16.json", "fp32": "r06_pmc_kernels_fp32.json"}
# frame kernels per stage (rocprofv3 symbol substrings) for the PMC bytes
FRAME_KERNELS = {"prep_inpaint": ("mdx::k_prep(", "k_inp_"),  # (not the model's k_preprocess_s2d)
                 "clean": ("k_median3", "k_morph", "k_clean_stream"),
                 "moments": ("k_moments",), "crop": ("k_crop",)}


F16_KEY = 100  # conv_roofline(split_dtypes=True): fp16-operand launches of kernel k are keyed F16_KEY + k


def conv_roofline(extractor, raw, steps=3, dump=None, split_dtypes=False):
    """Time every conv launch of `steps` serial steps with HIP events on the
    launch stream (mdx_model_profile: events recorded by the model handle
    around each mdx_conv2d launch; a Winograd layer as its input transform,
    batched GEMM and output transform) and tag it with the kernel the library
    chose.  Returns {kernel id: [FLOP (executed; HBM bytes for the
    transforms), seconds, launches, ksplit]} per step; with split_dtypes
    (config 5's fp32 trunk + fp16 heads) the fp16-operand launches of kernel
    k are counted under F16_KEY + k, so each is priced at its own peak."""
    import torch
    model = extractor.predictor.model
    rec = []
    model.profile(True)
    try:
        for _ in range(steps):
            extractor.step_device(raw)
            torch.cuda.synchronize()
            rec.extend(model.profile_read())
    finally:
        model.profile(False)
    per = {}
    for kid, ks, M, N, K, fl, ms, dt in rec:
        if split_dtypes and dt == 1:
            kid = F16_KEY + kid
        d = per.setdefault(kid, [0.0, 0.0, 0, 0])
        d[0] += fl / steps
        d[1] += ms * 1e-3 / steps
        d[2] += 1.0 / steps
        d[3] = max(d[3], ks)
    if dump:
        n = len(rec) // steps
        rows = [{"M": M, "N": N, "K": K, "kernel": kid, "ksplit": ks, "dtype": "fp16" if dt == 1 else "fp32",
                 "us": ms * 1e3, "tflops": fl / (ms * 1e-3) / 1e12 if ms > 0 else None}
                for kid, ks, M, N, K, fl, ms, dt in rec[-n:]]
        with open(dump, "w") as fh:
            json.dump(rows, fh, indent=0)
    return per


def _pmc(dtype):
    path = os.path.join(ROOT, "profiles", PMC_FILE[dtype])
    try:
        with open(path) as fh:
            return json.load(fh)["kernels"]
    except Exception:
        return {}


def _pmc_bytes(kern, sym):
    """PMC HBM bytes per launch of a kernel symbol; for a tuple of instances
    (the Winograd transforms of both tile sizes) the launch-weighted mean."""
    if isinstance(sym, tuple):
        recs = [kern.get(s) or kern.get(KERNEL_DEMANGLED.get(s, ""), {}) for s in sym]
        recs = [r for r in recs if r.get("hbm_bytes_per_launch") is not None]
        n = sum(r.get("launches_per_step", 0) for r in recs)
        return sum(r["hbm_bytes_per_launch"] * r.get("launches_per_step", 0) for r in recs) / n if n else None
    rec = kern.get(sym) or kern.get(KERNEL_DEMANGLED.get(sym, ""), {})
    return rec.get("hbm_bytes_per_launch")


def roofline_line(per, dtype, model_flop_per_step):
    """Roofline object for the dominant MFMA kernel: the one with the most GPU
    time per serial step (a Winograd layer's batched GEMM counts under the
    kernel it ran on, at its executed FLOPs).  `kernels` lists the top
    kernels by time; the transforms are HBM-bound and listed in GB/s."""
    from moseq2_detectron_extract_amd._lib import call, policy
    peak = PEAK[dtype]
    kern = _pmc(dtype)
    mfma = [k for k in per if k not in TRANSFORMS and k < F16_KEY]
    ranked = sorted(per, key=lambda k: -per[k][1])
    key = max(mfma, key=lambda k: per[k][1])
    fl, sec, n, ks = per[key]
    ach = fl / sec / 1e12
    sym = KERNEL_SYMBOLS[dtype].get(key)
    traffic = _pmc_bytes(kern, sym) if sym else None

    def row(k):
        f, t, c, _ = per[k]
        f16 = k >= F16_KEY  # an fp16-operand launch in a mixed-precision run: its own peak and symbol
        kb, dk = (k - F16_KEY, "fp16") if f16 else (k, dtype)
        r = {"kernel": KERNEL_NAMES.get(kb, str(kb)) + (" (fp16 operands)" if f16 else ""),
             "symbol": KERNEL_SYMBOLS[dk].get(kb), "launches_per_step": round(c), "ms_per_step": round(t * 1e3, 3)}
        if k in TRANSFORMS:
            r.update(gbytes_per_step=round(f / 1e9, 3), achieved_gbs=round(f / t / 1e9, 1),
                     frac_hbm=round(f / t / 1e9 / HBM_PEAK, 4))
        else:
            r.update(tflop_per_step=round(f / 1e12, 4), achieved_tflops=round(f / t / 1e12, 2),
                     frac=round(f / t / 1e12 / PEAK[dk], 4), peak=PEAK[dk])
        pb = _pmc_bytes(_pmc(dk) if f16 else kern, r["symbol"]) if r["symbol"] else None
        if pb is not None:
            r["pmc_hbm_bytes_per_launch"] = round(pb)
        return r

    mf = sum(v[0] for k, v in per.items() if k not in TRANSFORMS)
    tot_s = sum(v[1] for v in per.values())
    return {"bound": "mfma", "achieved": round(ach, 2), "peak": peak, "unit": "TFLOP/s",
            "frac": round(ach / peak, 4), "traffic": traffic,
            "kernel": f"{KERNEL_NAMES.get(key, key)} ({sym}): {n:.0f} launches/step, {fl / 1e12:.3f} executed "
                      f"TFLOP and {sec * 1e3:.3f} ms per step (HIP events on the launch stream, serial steps; "
                      f"achieved = executed FLOP / time; traffic = PMC HBM bytes per launch, profiles/{PMC_FILE[dtype]})",
            "kernels": [row(k) for k in ranked[:6]],
            "all_conv": {"launches": round(sum(v[2] for k, v in per.items() if k not in TRANSFORMS)),
                         "ms_per_step": round(tot_s * 1e3, 3),
                         "executed_tflop_per_step": round(mf / 1e12, 3),
                         "executed_tflops": round(mf / tot_s / 1e12, 1),
                         "model_tflop_per_step": round(model_flop_per_step / 1e12, 3),
                         "direct_equivalent_tflops": round(model_flop_per_step / tot_s / 1e12, 1),
                         "note": "time = every conv launch incl. the Winograd transforms; executed = the FLOPs the "
                                 "MFMA kernels perform (the Winograd GEMMs do 1/4 of the direct 3x3 FLOPs); "
                                 "direct_equivalent = the model's algorithmic FLOPs (direct convolution, heads "
                                 "included) over the same time, which can exceed the peak"},
            "winograd_tile": policy()["winograd"]}


def frame_ops_line(ex, raw, steps=5):
    """HBM roofline of the frame kernels: each stage of the frame path timed
    with HIP events on the issuing stream over `steps` repetitions, on one
    batch (the pipelined loop's launch: one workgroup per frame, so a 32-frame
    launch covers an eighth of the CUs) and on a 1024-frame chunk (the extract
    loop's launch: the batch tiled 32 times); algorithmic bytes per frame as
    SURVEY.md §8(d) counts them."""
    import torch
    from moseq2_detectron_extract_amd import proc
    kern = _pmc("fp32")

    def measure(raw_, reps):
        B, H, W = raw_.shape
        prepped, cleaned = ex.front(raw_)
        d2 = torch.cat([ex.infer(prepped[i:i + 32])["d2_mask"] for i in range(0, B, 32)])
        feats = proc.frame_moments(cleaned, d2, float(ex.cfg.frame_threshold))
        ang = torch.remainder(-torch.rad2deg(feats["orientation"]), 360)
        ch, cw = ex.cfg.crop_size
        px = prepped.shape[1] * prepped.shape[2]
        stages = {
            "prep_inpaint": (lambda: ex.prep(raw_), 2 * H * W + px),
            "clean": (lambda: proc.clean_frames(prepped, iters_tail=ex.cfg.iters_tail, strel_tail=ex.strel), 2 * px),
            "moments": (lambda: proc.frame_moments(cleaned, d2, float(ex.cfg.frame_threshold)), 2 * px),
            "crop": (lambda: ex.crop(prepped, d2, feats["centroid"], ang), 2 * 2 * ch * cw),
        }
        out, tb, tt = {}, 0.0, 0.0
        for name, (fn, bpf) in stages.items():
            fn()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize()
            e0.record()
            for _ in range(reps):
                fn()
            e1.record()
            torch.cuda.synchronize()
            t = e0.elapsed_time(e1) * 1e-3 / reps
            by = bpf * B
            tb += by
            tt += t
            r = {"us": round(t * 1e6, 1), "algorithmic_bytes_per_frame": bpf,
                 "achieved_gbs": round(by / t / 1e9, 1), "frac_hbm": round(by / t / 1e9 / HBM_PEAK, 4)}
            if B == 32:
                pm = [v["hbm_bytes_per_launch"] * v["launches_per_step"] for k, v in kern.items()
                      if any(sub in k for sub in FRAME_KERNELS[name])]
                if pm:
                    r["pmc_hbm_bytes"] = round(sum(pm))
            out[name] = r
        out["total"] = {"us": round(tt * 1e6, 1), "algorithmic_bytes_per_frame": round(tb / B),
                        "achieved_gbs": round(tb / tt / 1e9, 1), "frac_hbm": round(tb / tt / 1e9 / HBM_PEAK, 4)}
        return out

    res = {"batch_32": measure(raw, steps), "chunk_1024": measure(raw.repeat(32, 1, 1), 2)}
    res["note"] = ("HIP events on the issuing stream, serial; algorithmic bytes per SURVEY.md section 8(d); "
                   f"pmc = FETCH_SIZE x2 + WRITE_SIZE per 32-frame batch (profiles/{PMC_FILE['fp32']}); the "
                   "frame kernels are latency-bound (one workgroup per frame, inpaint / contour following "
                   "sequential inside a frame), not HBM-bound")
    return res


def extract_loop(args):
    """BASELINE config 3: extract.extract_session over a synthetic session
    written as depth.dat (frame source -> device path -> instance selection ->
    native Kalman / flip step -> scalars, keypoint tables, crops -> result
    writers), fp32, tracking on.  Disk write of the session is outside the
    timed region; reading it is inside."""
    import tempfile
    import torch
    from moseq2_detectron_extract_amd import synth
    from moseq2_detectron_extract_amd.extract import extract_session
    from moseq2_detectron_extract_amd.model import ModelConfig, Predictor
    from moseq2_detectron_extract_amd.pipeline import ExtractConfig
    n, chunk = args.extract_frames, args.extract_chunk
    workers = max(1, min(16, len(os.sched_getaffinity(0)), int(os.environ.get("OMP_NUM_THREADS", 16))))
    s = synth.SyntheticSession(n, seed=9)
    pred = Predictor.from_config(ModelConfig(depth=args.depth, score_thresh_test=0.0), weights="synthetic")
    cfg = ExtractConfig(chunk_size=chunk, use_tracking=True, stream_chunks=not args.extract_per_chunk)
    with tempfile.TemporaryDirectory(dir=os.environ.get("TMPDIR", "/tmp")) as td:
        t0 = time.perf_counter()
        s.write(td, workers=workers)
        write_s = time.perf_counter() - t0
        path = os.path.join(td, "depth.dat")
        # warm-up over the first chunk (plans, workspaces, allocator pools)
        extract_session(path, s.bground_im, s.roi, pred, cfg, true_depth=s.true_depth, frame_trim=(0, n - chunk))
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        out = extract_session(path, s.bground_im, s.roi, pred, cfg, true_depth=s.true_depth,
                              output_dir=os.path.join(td, "out"))
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        written = sorted(os.listdir(os.path.join(td, "out")))
    assert out["frames"].shape[0] == n
    return {"value": round(n / dt, 2), "unit": "frames/s", "seconds": round(dt, 3), "dtype": pred.model.dtype,
            "config": f"{n} frames, chunks of {chunk}, use_tracking=True, R{args.depth}-FPN, batch "
                      f"{cfg.batch_size}, {cfg.model_streams} model streams",
            "written": written, "session_write_s": round(write_s, 1),
            "note": "extract.extract_session (M/extract.py:22-139 without its control plane): .dat reads (page "
                    "cache), prep+inpaint, R-CNN forward, mask NMS, instance selection (norfair semantics), "
                    "clean, moments, native Kalman/flip angle step (host thread beside the next chunk's device "
                    "pass), scalars, keypoint tables, crops, results + keypoints TSV writers"}


def cpu_baseline(nframes: int, dtype_cfg, chunk: int = 16):
    """Oracle (CPU restatement of the reference path) timed on the host
    cores: prep + NS inpaint (C), scale, PyTorch-CPU fp32 Mask/Keypoint R-CNN
    forward with torchvision's roi_align / nms kernels in C (model_ops.c),
    mask NMS + instance 0, clean / moments / crop (C).  Frames go through in
    chunks of `chunk`."""
    import numpy as np
    import torch
    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd import synth
    from moseq2_detectron_extract_amd.model import synthetic_state_dict
    from oracle import features_ref as FR
    from oracle import frameops as O
    from oracle import model_ref as R
    cores = len(os.sched_getaffinity(0))
    # the GPU box exposes the whole machine's cores but grants this job a share
    # (OMP_NUM_THREADS); oversubscribing 256 threads is far slower
    cores = min(cores, int(os.environ.get("OMP_NUM_THREADS", cores)))
    torch.set_num_threads(cores)
    os.environ["OMP_NUM_THREADS"] = str(cores)  # model_ops.c's OpenMP pool
    s = synth.SyntheticSession(nframes, seed=123)
    raw = s.frames(0, nframes)
    sd = synthetic_state_dict(dtype_cfg, 0)
    R.forward(sd, dtype_cfg, O.scale_raw_frames(O.prep_raw_frames(raw[:1], s.bground_im, s.roi, 0, 100)[0], 0,
                                                 100)[..., None], keep_intermediates=False)  # warm-up
    t0 = time.perf_counter()
    for a in range(0, nframes, chunk):
        r = raw[a:a + chunk]
        prepped, _ = O.prep_raw_frames(r, s.bground_im, s.roi, 0, 100)
        scaled = O.scale_raw_frames(prepped, 0, 100)
        res, _ = R.forward(sd, dtype_cfg, scaled[..., None], keep_intermediates=False)
        d2 = np.zeros(prepped.shape, np.uint8)
        for i, rr in enumerate(res):
            keep = FR.nms_mask_instances(rr["pred_masks"].numpy(), rr["scores"].numpy())
            if keep:
                d2[i] = rr["pred_masks"][keep[0]].numpy()
        cl = O.clean_frames(prepped, iters_tail=3)
        f = O.get_frame_features(cl, 3, mask=d2)
        ang = np.mod(-np.rad2deg(f["orientation"]), 360)
        O.crop_and_rotate_frames(prepped, f["centroid"], ang)
        O.crop_and_rotate_frames(d2, f["centroid"], ang)
    dt = time.perf_counter() - t0
    return {"value": nframes / dt, "unit": "frames/s", "cores": cores, "kind": "port",
            "sample": f"{nframes} synthetic 512x424 frames in chunks of {chunk} through the CPU oracle (C prep + NS "
                      f"inpaint, PyTorch-CPU fp32 R50-FPN Mask/Keypoint R-CNN with torchvision's roi_align/nms "
                      f"restated in C, mask NMS, C clean/moments/crop; SCORE_THRESH_TEST=0), {dt:.1f} s"}


def measure(args, dtype, B, world, rank, raw_host, sess, dist, gather_bufs, depth=None):
    """Warm up, then time args.steps batches of the overlapped hot path with
    the H2D copy of every raw batch from pinned host memory inside the timed
    region.  Returns (seconds (max over ranks), extractor)."""
    import torch
    from moseq2_detectron_extract_amd.model import ModelConfig, Predictor
    from moseq2_detectron_extract_amd.pipeline import ExtractConfig, GPUExtractor, OverlappedExtractor
    cfg = ModelConfig(depth=depth or args.depth, score_thresh_test=0.0)
    pred = Predictor.from_config(cfg, dtype=dtype, seed=0, weights="synthetic")
    ns = 1 if args.no_overlap else max(1, args.model_streams)
    ex = GPUExtractor(sess.bground_im, sess.roi, pred, ExtractConfig(batch_size=B, model_streams=ns))
    pipe = OverlappedExtractor(ex, ns) if args.pipeline and not args.no_overlap else None
    # default (chunked) loop: the reference's InferenceStep shape -- a chunk of
    # --chunk-batches batches is prepped / inpainted / cleaned, its
    # batch_size-frame forwards alternate over ns streams (GPUExtractor.infer;
    # the streams drift apart, so the forwards overlap out of phase), then the
    # chunk's moments / crops; `step` stays one 32-frame batch
    chunk = 1 if pipe is not None else (max(1, args.chunk_batches) if ns > 1 else 1)
    gstream = torch.cuda.Stream() if world > 1 else None
    h2d = torch.cuda.Stream()
    # the loop issues from a pool stream, not HIP's legacy NULL stream: an
    # event recorded on the NULL stream also waits for all earlier work of
    # every blocking stream, which would order each front behind the
    # previous forward
    issue_stream = torch.cuda.Stream()
    resident = None if not args.no_h2d else [t.cuda() for t in raw_host]

    def deliver(r):
        if r is not None and world > 1:
            # on a side stream, so the hand-off never orders the caller's
            # stream (and the pipeline's next fronts) behind this batch
            if "ready" not in r:  # chunked loop: the results were produced on the issuing stream
                ev = torch.cuda.Event()
                ev.record(torch.cuda.current_stream())
                r = dict(r, ready=ev)
                for k in ("depth_frames", "mask_frames"):
                    r[k].record_stream(gstream)
            with torch.cuda.stream(gstream):
                gstream.wait_event(r["ready"])
                payload = torch.stack([r["depth_frames"], r["mask_frames"]], 1).contiguous()
                if gather_bufs is not None and payload.shape[0] != gather_bufs[0].shape[0]:
                    gather_bufs[:] = [torch.empty_like(payload, device=gather_bufs[0].device) for _ in gather_bufs]
                if gather_bufs is not None and gather_bufs[0].device.type == "cpu":
                    payload = payload.cpu()
                dist.gather(payload, gather_bufs if rank == 0 else None, dst=0)

    def upload(i, n=1):
        # batches i .. i+n-1 (the two pinned host batches alternate)
        if resident is not None and n == 1:
            return resident[i % 2]
        shape = (n * raw_host[0].shape[0],) + tuple(raw_host[0].shape[1:])
        with torch.cuda.stream(h2d):
            raw = torch.empty(shape, dtype=raw_host[0].dtype, device="cuda")
            for q in range(n):
                src = raw_host[(i + q) % 2] if resident is None else resident[(i + q) % 2]
                raw[q * B:(q + 1) * B].copy_(src, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(h2d)
        issue_stream.wait_event(ev)
        raw.record_stream(issue_stream)
        return raw

    def run(nsteps, offset):
        # nsteps batches through the path; with the pipeline the last batch is
        # flushed inside, so exactly nsteps batches complete
        with torch.cuda.stream(issue_stream):
            i = 0
            while i < nsteps:
                n = min(chunk, nsteps - i)
                raw = upload(offset + i, n)
                deliver(ex.step_device(raw) if pipe is None else pipe.submit(raw))
                i += n
            if pipe is not None:
                for r in pipe.flush():
                    deliver(r)

    if pipe is not None:
        pipe.prime(raw_host[0].cuda())
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
        t = torch.tensor([dt], dtype=torch.float64,
                         device="cpu" if dist.get_backend() == "gloo" else "cuda")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
    return dt, ex, cfg


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    # MDX_BENCH_BACKEND=gloo rehearses the multi-rank path with every rank on
    # the one GPU of a test box (the driver's runs use nccl = RCCL, one GPU each)
    backend = os.environ.get("MDX_BENCH_BACKEND", "nccl")
    dev = local % max(1, torch.cuda.device_count()) if backend == "gloo" else local
    if world > 1:
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", dev))
        else:
            dist.init_process_group(backend)
    torch.cuda.set_device(dev)

    import mdx_pkg
    mdx_pkg.load()
    from moseq2_detectron_extract_amd import synth
    from moseq2_detectron_extract_amd.model import ModelConfig
    from moseq2_detectron_extract_amd.model.runtime import flops_per_image

    from moseq2_detectron_extract_amd._lib import POLICY_FIELDS, set_policy
    upd = {k: v for k, v in (("dma_f32", args.dma_f32), ("winograd", args.winograd),
                             ("winograd_min_cin", args.winograd_min_cin), ("roi_mode", args.roi_mode)) if v is not None}
    for kv in args.set:
        field, val = kv.split("=")
        if field not in POLICY_FIELDS:
            raise SystemExit(f"--set: {field} is not a field of mdx_policy ({', '.join(POLICY_FIELDS)})")
        upd[field] = int(val)
    if upd:
        set_policy(**upd)
    B = args.batch
    sess = synth.SyntheticSession(2 * B, seed=1000 + rank)
    frames = sess.frames(0, 2 * B)
    raw_host = [torch.from_numpy(frames[i * B:(i + 1) * B]).pin_memory() for i in range(2)]
    gather_bufs = None
    if world > 1:
        gdev = "cpu" if backend == "gloo" else "cuda"
        gather_bufs = [torch.empty((B, 2, 80, 80), dtype=torch.uint8, device=gdev) for _ in range(world)]

    dt, ex, cfg = measure(args, args.dtype, B, world, rank, raw_host, sess, dist, gather_bufs)
    frames_done = world * args.steps * B
    value = frames_done / dt

    roof = None
    if not args.no_roofline:
        raw_dev = raw_host[0].cuda()
        per = conv_roofline(ex, raw_dev, dump=args.dump_convs, split_dtypes=args.dtype == "mixed")
        roof = roofline_line(per, "fp32" if args.dtype == "mixed" else args.dtype, flops_per_image(cfg) * B)
        roof["frame_ops"] = frame_ops_line(ex, raw_dev)
    del ex
    torch.cuda.synchronize()

    secondary = None
    if not args.no_secondary and args.dtype == "fp32":
        dt16, ex16, cfg16 = measure(args, "fp16", B, world, rank, raw_host, sess, dist, gather_bufs)
        secondary = {"fp16": {"value": round(frames_done / dt16, 2), "unit": "frames/s",
                              "ms_per_step": round(dt16 / args.steps * 1e3, 3), "dtype": "fp16",
                              "note": "fp16 MFMA forward (fp32 accumulation), same loop; tolerance vs the fp32 "
                                      "oracle: tests/test_parity_full.py::test_forward_full_frame[50-32-fp16-0-0]"}}
        if not args.no_roofline:  # its own roofline: the dominant fp16 kernel at the dense fp16 peak
            per16 = conv_roofline(ex16, raw_host[0].cuda())
            r16 = roofline_line(per16, "fp16", flops_per_image(cfg16) * B)
            secondary["fp16"]["roofline"] = {k: r16[k] for k in ("bound", "achieved", "peak", "unit", "frac", "traffic",
                                                                 "kernel", "kernels", "all_conv")}
        del ex16
    if not args.no_secondary and args.dtype == "fp32" and not args.no_x6:
        torch.cuda.synchronize()
        from moseq2_detectron_extract_amd._lib import policy_scope
        with policy_scope(fp32_split=6):  # the handle measure() creates captures it
            dtx, exx, _ = measure(args, "fp32", B, world, rank, raw_host, sess, dist, gather_bufs)
        secondary["fp32_bf16x6"] = {
            "value": round(frames_done / dtx, 2), "unit": "frames/s", "ms_per_step": round(dtx / args.steps * 1e3, 3),
            "dtype": "fp32 operands split exactly into 3 bf16 planes, 6 plane products on the bf16 matrix cores, "
                     "fp32 accumulation",
            "note": "mdx_policy.fp32_split = 6: conv layers and Winograd GEMMs on k_conv_x3 (weights split into "
                    "planes once when the handle is created, activations split in registers), box head FCs on "
                    "k_gemm_x6 (256x256 LDS-DMA over planes written by the box pooler / mdx_split_x6); per product the "
                    "dropped terms are below one fp32 rounding; "
                    "full-frame parity vs the fp32 oracle at least as close as the f32-MFMA kernels' "
                    "(tests/test_parity_full.py::test_forward_full_frame[50-32-fp32-4-6] and [50-32-fp32-6-6], "
                    "DESIGN.md section 3)"}
        del exx

    if not args.no_secondary and not args.no_config5 and args.dtype == "fp32" and args.depth == 50:
        # BASELINE config 5 as stated: R101-FPN, batch 64, fp32 trunk / RPN /
        # box head with the keypoint + mask heads in fp16 ("mixed"), the same
        # loop, its own roofline
        torch.cuda.synchronize()
        secondary = secondary or {}
        try:
            B5 = 64
            sess5 = synth.SyntheticSession(2 * B5, seed=2000 + rank)
            f5 = sess5.frames(0, 2 * B5)
            raw5 = [torch.from_numpy(f5[i * B5:(i + 1) * B5]).pin_memory() for i in range(2)]
            gb5 = None if gather_bufs is None else \
                [torch.empty((B5, 2, 80, 80), dtype=torch.uint8, device=gather_bufs[0].device) for _ in range(world)]
            dt5, ex5, cfg5 = measure(args, "mixed", B5, world, rank, raw5, sess5, dist, gb5, depth=101)
            c5 = {"value": round(world * args.steps * B5 / dt5, 2), "unit": "frames/s",
                  "ms_per_step": round(dt5 / args.steps * 1e3, 3), "dtype": "mixed",
                  "config": {"workload": "BASELINE config 5: R101-FPN Mask/Keypoint R-CNN, batch 64, fp32 backbone / "
                                         "FPN / RPN / box head, fp16 mask + keypoint heads, same hot path and loop",
                             "global_batch": B5 * world, "model_gflop_per_frame": round(flops_per_image(cfg5) / 1e9, 2)},
                  "note": "parity: tests/test_parity_full.py::test_forward_full_frame[101-64-mixed-6-0]"}
            if not args.no_roofline:
                per5 = conv_roofline(ex5, raw5[0].cuda(), split_dtypes=True)
                r5 = roofline_line(per5, "fp32", flops_per_image(cfg5) * B5)
                c5["roofline"] = {k: r5[k] for k in ("bound", "achieved", "peak", "unit", "frac", "kernel", "kernels",
                                                     "all_conv")}
            secondary["config5"] = c5
            del ex5
        except Exception as e:  # a secondary must never sink the bench line
            secondary["config5"] = {"value": None, "error": repr(e)[:300]}

    if world == 1 and not args.no_secondary and not args.no_extract_loop and args.dtype == "fp32":
        torch.cuda.synchronize()
        secondary = secondary or {}
        try:
            secondary["extract_loop"] = extract_loop(args)
        except Exception as e:  # a secondary must never sink the bench line
            secondary["extract_loop"] = {"value": None, "error": repr(e)[:300]}

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
            "config": {"workload": f"full extract hot path ({'pinned-host H2D, ' if not args.no_h2d else ''}"
                                   f"prep+inpaint, scale, R{args.depth}-FPN Mask/Keypoint R-CNN {args.dtype}, mask "
                                   f"NMS, clean, moments, crop), 512x424 int16 frames",
                       "global_batch": B * world, "per_gpu_batch": B, "frame": [424, 512],
                       "model_gflop_per_frame": round(flops_per_image(cfg) / 1e9, 2),
                       "parallelism": f"frame-sharded x{world}",
                       "h2d_in_timed_region": not args.no_h2d,
                       "gpu_max_hw_queues": os.environ.get("GPU_MAX_HW_QUEUES"),
                       "streams": "1" if args.no_overlap else (
                           f"{3 + args.model_streams} (H2D, prep/inpaint/clean of the newest batch, "
                           f"{args.model_streams} model forwards + mask selection of the next batches, moments/crop "
                           f"of the oldest)" if args.pipeline else
                           f"chunks of {args.chunk_batches} batches: H2D on its own stream, prep/inpaint/clean of "
                           f"the chunk, its forwards + mask selection alternating over {args.model_streams} "
                           f"streams, moments/crop of the chunk")},
            "roofline": roof, "cpu_baseline": cpu, "secondary": secondary,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
