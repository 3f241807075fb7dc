/*
 * mdx.h -- C ABI of the MI355X-native moseq2-detectron-extract hot path.
 *
 * Every entry point takes plain device pointers + sizes and an optional HIP
 * stream (mdx_stream_t == hipStream_t, NULL = default stream).  The caller owns
 * every input/output buffer (PyTorch-ROCm allocates them); the library only
 * allocates workspace it owns through a handle.  All work is enqueued on the
 * given stream; no entry point synchronises the host unless its comment says
 * so.  Return value: 0 on success, a negative MDX_E* code on failure, with a
 * thread-local message in mdx_last_error().
 *
 * Each function cites the reference interface it replaces
 * (M/ = moseq2_detectron_extract/ in tischfieldlab/moseq2-detectron-extract).
 */
#ifndef MDX_H_
#define MDX_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef void *mdx_stream_t; /* hipStream_t */

enum {
    MDX_OK = 0,
    MDX_EINVAL = -1,   /* bad argument / shape */
    MDX_EHIP = -2,     /* HIP runtime error */
    MDX_ENOMEM = -3,   /* workspace allocation failed */
    MDX_ELIMIT = -4    /* input exceeds a compiled-in limit */
};

/* Thread-local text of the last error ("" when none). */
const char *mdx_last_error(void);
/* Library version string, e.g. "mdx 0.1.0 gfx950". */
const char *mdx_version(void);

/* ---------------------------------------------------------------------
 * Frame ops (M/proc/proc.py)
 * ------------------------------------------------------------------- */

/* prep_raw_frames(frames, bground_im, roi, vmin, vmax, 'uint8',
 *                 fix_invalid_pixels) -- numpy part.  M/proc/proc.py:129-172,
 * find_invalid_pixels :175-186, apply_roi/get_bbox M/proc/roi.py:215-254.
 * raw      int16 [n][H][W]
 * bg       float64 [H][W] or NULL (no background subtraction)
 * roi      uint8 [H][W] 0/1 or NULL (no masking); [y0,y1)x[x0,x1) is the
 *          crop (get_bbox max is exclusive, reference quirk)
 * flags    bit0: vmin given, bit1: vmax given
 * out      uint8 [n][y1-y0][x1-x0]
 * invalid  uint8 [n][y1-y0][x1-x0] or NULL: (raw==0)*roi, cropped */
int mdx_prep_frames(const int16_t *raw, int64_t n, int H, int W, const double *bg,
                    const uint8_t *roi, int y0, int y1, int x0, int x1, int flags,
                    double vmin, double vmax, uint8_t *out, uint8_t *invalid,
                    mdx_stream_t stream);

/* fill_invalid_pixels -> cv2.inpaint(frame, invalid, 3, cv2.INPAINT_NS) per
 * frame, in place on `frames`.  M/proc/proc.py:189-210.  workspace: device
 * buffer of at least mdx_inpaint_workspace_bytes(n, H, W) bytes, set up once
 * by mdx_inpaint_workspace_init for frames of H x W (and again before it is
 * used for another frame shape); every call leaves it ready for the next.
 * Per frame it holds mdx_inpaint_sparse_capacity(H, W) unknown pixels (about
 * 4 % of the frame; < 1 MB per 512 x 424 frame); frames with more unknown
 * pixels are done one after another in one shared full-size slot.  A call on a
 * workspace not set up for H x W leaves the frames un-inpainted, counts each
 * of them in mdx_inpaint_errors / `errors`, and the workspace must be set up
 * again before its next use. */
int64_t mdx_inpaint_workspace_bytes(int64_t n, int H, int W);
int mdx_inpaint_workspace_init(void *workspace, int64_t bytes, int H, int W, mdx_stream_t stream);
int mdx_inpaint_sparse_capacity(int H, int W);
int mdx_inpaint_ns(uint8_t *frames, const uint8_t *invalid, int64_t n, int H, int W,
                   int radius, void *workspace, mdx_stream_t stream);
/* Frames whose inpaint cluster labelling failed its convergence check (every
 * label must be its own root before the labels index the cluster tables) since
 * the last reset; such a frame is left un-inpainted.  Synchronous (reads a
 * device counter); reset != 0 clears it.  Expected 0: tests assert it. */
int mdx_inpaint_errors(int reset);
/* mdx_inpaint_ns that also adds its unconverged frames to the caller's device
 * counter `errors` (one uint32, stream-ordered): a per-session count that
 * other users of the library in the same process do not touch.  NULL = the
 * process-wide counter only. */
int mdx_inpaint_ns_counted(uint8_t *frames, const uint8_t *invalid, int64_t n, int H, int W, int radius,
                           void *workspace, unsigned int *errors, mdx_stream_t stream);
/* prep_raw_frames with fix_invalid_pixels=True in one call: mdx_prep_frames
 * (invalid may be NULL: the invalid pixels then go to the workspace only, as
 * a bit image) followed by the inpaint of `out` with `radius`.  workspace: as
 * for mdx_inpaint_ns, for frames of (y1 - y0) x (x1 - x0).
 * M/proc/proc.py:129-172 + 189-210. */
int mdx_prep_inpaint(const int16_t *raw, int64_t n, int H, int W, const double *bg, const uint8_t *roi,
                     int y0, int y1, int x0, int x1, int flags, double vmin, double vmax, uint8_t *out,
                     uint8_t *invalid, int radius, void *workspace, unsigned int *errors, mdx_stream_t stream);

/* scale_raw_frames(frames, vmin, vmax, 'uint8') as a 256-entry LUT built on
 * the host in float64 (M/proc/proc.py:214-234).  int_vmin != 0 reproduces
 * numpy's uint8 - int wraparound.  Host-only, no device work. */
int mdx_build_scale_lut(double vmin, double vmax, int int_vmin, uint8_t lut[256]);
/* out[i] = lut[in[i]] for count bytes (device pointers; lut is host). */
int mdx_scale_frames(const uint8_t *in, int64_t count, const uint8_t lut[256], uint8_t *out,
                     mdx_stream_t stream);

/* clean_frames(frames, prefilter_space=(median_k,), strel_tail=strel,
 * iters_tail=iters) -- M/proc/proc.py:480-515: per frame medianBlur(median_k)
 * (0 = skip; only 3 supported) then morphologyEx(MORPH_OPEN, strel, iters).
 * strel: host uint8 [kh][kw] (each row one contiguous run, kh,kw <= 15).
 * src, out and workspace (mdx_clean_workspace_bytes; unused when iters == 0)
 * must not alias. */
int64_t mdx_clean_workspace_bytes(int64_t n, int H, int W);
int mdx_clean_frames(const uint8_t *src, int64_t n, int H, int W, int median_k,
                     const uint8_t *strel, int kh, int kw, int iters, uint8_t *out,
                     uint8_t *workspace, mdx_stream_t stream);
/* clean_frames kernel choice: 0 = one launch per pass, 1 = the fused streaming
 * kernel with the strip width chosen by batch size (default), 2 = 256-column
 * strips, 3 = 512-column strips.  The fused kernel serves median 3 + opening
 * with the 9x9 ellipse, 3 iterations (the extract path); other parameters run
 * the per-pass kernels.  Returns the previous mode. */
int mdx_clean_set_mode(int mode);

/* get_frame_features(frames, frame_threshold=thr, mask=mask, use_cc=*) +
 * im_moment_features -- M/proc/proc.py:237-302, :518-549.  Largest contour
 * (findContours RETR_TREE + contourArea argmax) and its polygon moments.
 * mask may be NULL.  Outputs (float64, NaN when no contour):
 * centroid [n][2] (x, y), orientation [n] (rad), axis_length [n][2],
 * area [n] (contourArea of the chosen contour; may be NULL). */
int mdx_frame_moments(const uint8_t *frames, const uint8_t *mask, int64_t n, int H, int W,
                      double thr, double *centroid, double *orientation, double *axis_length,
                      double *area, mdx_stream_t stream);
/* mdx_frame_moments with a caller workspace of
 * mdx_frame_moments_workspace_bytes(n, H, W) bytes: the threshold / mask
 * bit-packing runs as its own launch over every CU (one wave per 64 pixels),
 * the contour following per frame reads the packed words (the path the
 * Python layer takes).  workspace NULL = packing inside the per-frame
 * kernel. */
int64_t mdx_frame_moments_workspace_bytes(int64_t n, int H, int W);
int mdx_frame_moments_ws(const uint8_t *frames, const uint8_t *mask, int64_t n, int H, int W, double thr,
                         double *centroid, double *orientation, double *axis_length, double *area,
                         void *workspace, mdx_stream_t stream);

/* crop_and_rotate_frame(frame, center, angle, crop_size=(cw, ch)) for every
 * frame of src0 (and of src1 when not NULL, same centers/angles) --
 * M/proc/proc.py:305-340, called twice per frame at
 * M/pipeline/process_features_step.py:186-198.
 * center float64 [n][2] (x, y), angle_deg float64 [n]; out uint8 [n][ch][cw].
 * window int32 [n][4] or NULL: the integer crop window (xmin, xmax, ymin,
 * ymax) in the zero-bordered frame, computed as the reference does
 * (int() truncation, proc.py:325-328); -1 x4 for frames the reference
 * returns zeros for before computing one (NaN angle / centre, centre < 0). */
int mdx_crop_rotate(const uint8_t *src0, const uint8_t *src1, int64_t n, int H, int W,
                    const double *center, const double *angle_deg, int cw, int ch,
                    uint8_t *out0, uint8_t *out1, int32_t *window, mdx_stream_t stream);


/* Per-frame reductions of compute_scalars (M/proc/scalars.py:79-103) over
 * frames * masks (uint8 product, M/pipeline/process_features_step.py:165):
 * area_px[i] = #{p : min_height < v < max_height}, height_ave[i] = mean of
 * those v (0 when none).  masks may be NULL (all ones).  With K > 0 also the
 * keypoint z lookup of keypoints_to_dict (M/proc/keypoints.py:122-130):
 * z_data[i][k] = z_frames[i][clip(floor(y))][clip(floor(x))] for keypoints
 * float64 [n][K][3] (NaN -> index 0, numpy's cast).  area_px int64 [n],
 * height_ave / z_data float64. */
int mdx_frame_scalars(const uint8_t *frames, const uint8_t *masks, int64_t n, int H, int W,
                      double min_height, double max_height, const double *keypoints, int K,
                      const uint8_t *z_frames, int64_t *area_px, double *height_ave, double *z_data,
                      mdx_stream_t stream);

/* Session background, get_bground_im M/proc/roi.py:293-307
 * as find_roi calls it (M/io/session.py:212-213): every frame int16 [n][H][W]
 * is median-blurred (cv2.medianBlur, BORDER_REPLICATE, med_scale 3 or 5) into
 * `work` (int16, n*H*W, caller-owned), then out[H][W] (float64) =
 * np.median(work, axis=0): the middle value, or the mean of the two middle
 * values for even n; NaN when n == 0.  n <= 65535. */
int mdx_bground_median(const int16_t *frames, int64_t n, int H, int W, int med_scale, int16_t *work,
                       double *out, mdx_stream_t stream);

/* Host (CPU) function: iterative_filter_angles (M/proc/proc.py:627-654) over
 * float64 angles[n] with the moving median of filter_angles (:600-624,
 * bottleneck move_median, min_count 1): repeat until np.allclose(curr, last)
 * or max_iters; out[n] the filtered angles, flips[n] = isclose(|out - in|,
 * 180).  Bit-identical to the numpy code; runs without the GIL. */
int mdx_iterative_filter_angles(const double *angles, int64_t n, int window, double tolerance, int max_iters,
                                double *out, uint8_t *flips);

/* Host (CPU) function: flips_from_keypoints (M/proc/proc.py:851-889): per
 * frame, keypoints float64 [n][K][3] (K >= 7; 0-3 front, 4-6 rear) rotated
 * by -angle_deg about centroid [n][2] vote for the end of the body axis
 * (centroid x -+ length / 2) they are nearer to; flips[n] = front mean vote
 * < rear mean vote, conf[n] = share of the 7 votes agreeing with it. */
int mdx_flips_from_keypoints(const double *kp, int64_t n, int K, const double *centroid,
                             const double *angle_deg, const double *length, uint8_t *flips, double *conf);

/* Keypoints TSV rows as ResultWriterStep writes them with pandas'
 * DataFrame.to_csv(sep="\t", index=False) (M/pipeline/write_results_step.py:
 * 54-73): columns cols[c] of nrows values, kinds[c] 0 float64 (Python repr,
 * NaN as an empty field), 1 bool (uint8: True / False), 2 int64; rows end in
 * '\n', no header.  Host code (no GPU): returns the bytes written into out
 * (cap >= nrows * (ncols * 40 + 1)), or a negative error. */
int64_t mdx_format_tsv_rows(const void *const *cols, const int *kinds, int ncols, int64_t nrows, char *out,
                            int64_t cap);

/* Host (CPU) function: the no-tracking angle branch of instances_to_features
 * (M/proc/proc.py:720-724, 827-839): angle = clamp_angles_deg(-rad2deg(
 * orientation)); +180 where mdx_flips_from_keypoints (length = max axis)
 * flips; iterative_filter_angles(window 3, tolerance 60, 1000 iterations);
 * flips_out = keypoint flips xor filter flips.  float64 in, angles_out
 * float64 [n], flips_out uint8 [n]. */
int mdx_finalize_angles(const double *orientation, const double *axis_length, const double *centroid,
                        const double *kp, int64_t n, int K, double *angles_out, uint8_t *flips_out);

/* Host (CPU) functions: the tracking branch of instances_to_features
 * (--use-tracking, the reference's default; M/proc/proc.py:720-800) with
 * ProcessFeaturesStep's point tracker (centroid + K keypoints, order-3
 * Kalman items) and angle tracker ((sin, cos), order 3)
 * (M/pipeline/process_features_step.py:40-51, M/proc/kalman.py:101-418),
 * pykalman semantics: EM (10 iterations on Q, R, P0) on the first chunk,
 * RTS smoothing per chunk (state carried), keypoint flips, alignment
 * scores and the per-frame sample / intervene / filter_update angle loop.
 * track: centroid [n][2], keypoints [n][K][3], orientation [n] (rad),
 * axis_length [n][2] (float64) -> smoothed centroid, keypoints (first 7
 * smoothed), angles (deg), flips.  state: which 0 = point, 1 = angle
 * tracker; *initialized, and its last state mean (returns its length). */
void *mdx_tracking_create(int n_keypoints);
int mdx_tracking_destroy(void *handle);
int mdx_tracking_state(void *handle, int which, int *initialized, double *mean, int64_t mean_len);
int mdx_tracking_track(void *handle, int64_t n, int K, const double *centroid, const double *keypoints,
                       const double *orientation, const double *axis_length, double *centroid_out,
                       double *keypoints_out, double *angles_out, uint8_t *flips_out);

/* Host (CPU) functions: the instance tracker of
 * ProcessFeaturesStep.__select_instances (M/pipeline/process_features_step.py:
 * 35-38, 133-160; norfair 2.x Tracker semantics, see instances.py).  The
 * tracker state carries from call to call (chunks in session order).
 * select: per frame f < n, nkeep[f] kept detections with centres
 * centers[f][0..nkeep[f])[2] (row, col; rows of D) -> out_n[f] = -1 when the
 * frame's instances stay as they are, else the number picked (<=
 * expected_instances) with out_ids[f][m] = (session frame, kept slot) of
 * each pick, oldest object first.  frame0 = the session index of frame 0. */
void *mdx_instance_tracker_create(int expected_instances);
int mdx_instance_tracker_destroy(void *handle);
int mdx_instance_tracker_select(void *handle, const int *nkeep, const double *centers, int64_t n, int D,
                                int64_t frame0, int *out_n, int64_t *out_ids);

/* ---------------------------------------------------------------------
 * Mask/Keypoint R-CNN forward (Predictor.__call__, M/model/predict.py:53-102,
 * Detectron2 GeneralizedRCNN built by M/model/config.py:21-94).  Tensors are
 * NHWC; dtype codes: 0 = float32, 1 = float16 (fp32 accumulation).
 * ------------------------------------------------------------------- */

/* Kernel-selection policy of the model path (one struct instead of a setter
 * per knob; replaces nothing in the reference: Detectron2 / cuDNN pick their
 * algorithms internally).  The policy in force for a call is
 *   - inside mdx_model_reserve / mdx_model_forward (and the handle's other
 *     entry points): the model handle's own, captured from the creating
 *     thread's policy at mdx_model_create (the weights are packed for it:
 *     Winograd transforms, bf16 planes, folded stem, fused shortcuts);
 *   - otherwise (direct mdx_conv2d / mdx_conv3x3_winograd / mdx_roi_align /
 *     mdx_rpn_proposals calls): the calling thread's, set with
 *     mdx_policy_set (initially the library defaults, mdx_policy_defaults).
 * No process-global state: two handles with different policies run
 * concurrently on different streams or threads.  Defaults in brackets. */
typedef struct mdx_policy {
    /* fp32 3x3 stride-1 layers with Cin >= winograd_min_cin [64]: 0 direct,
     * 2 / 4 Winograd F(2x2,3x3) / F(4x4,3x3), 6 F(6x6,3x3) where
     * mdx_winograd_tile picks it and F(4x4,3x3) elsewhere [6] */
    int winograd, winograd_min_cin;
    /* Winograd GEMMs (Cout % 256 == 0) on the 256x256 LDS-DMA kernel: 0 never
     * [0: measured no faster], 1 from winograd_dma_min_wgs [384] workgroups,
     * 2 whenever eligible */
    int winograd_dma, winograd_dma_min_wgs;
    /* model handles: Winograd layers in image slices of at most this many MB
     * of transformed input, kept in the Infinity Cache between the three
     * launches; 0 = one pass [0] */
    int wino_slice_mb;
    /* fp32 layers as exact bf16 plane products: 0 the f32 MFMA kernels [0],
     * 6 the six largest of the nine plane products, 9 all nine */
    int fp32_split;
    /* split-plane launches: the 64-wide N tile everywhere [1]; the
     * single-stage instance with pre-split weights [1] */
    int x3_narrow, x3_single_stage;
    /* fp16 layers (Cin % 64 == 0) on the 256x256 LDS-DMA kernel: 0 never,
     * 1 when the layer fills the chip [1], 2 whenever eligible, 3 / 4 as 2 / 1
     * on the 256x128 tile */
    int large_tiles;
    /* fp16 layers on the 128x128 LDS-DMA kernel: 0 never [0: slower in the
     * full forward], 1 from dma128_min_tiles [1536] tiles, 2 whenever
     * eligible; its DMA pieces issued between the MFMAs [1] */
    int dma128, dma128_min_tiles, dma128_interleave;
    /* fp32 layers (Cin % 32 == 0) on the LDS-DMA kernels: 0 never [0: the
     * single-stage register-staged kernel is faster], 1 the 128x128 tile,
     * 2 the 256x256 tile for >= 500 tiles and K >= 1024, 3 the 256x256 tile
     * under the fp16 policy, 4 as 2 also in split-plane mode (diagnostic) */
    int dma_f32;
    /* pointwise layers on the instances with per-row load addresses [1] */
    int pointwise;
    /* single-LDS-stage instances: 1 fp32 pointwise, 2 + fp32 KxK, 3 + fp16
     * pointwise, 4 + fp16 KxK [4]; 0 the two-stage instances */
    int single_stage;
    /* fp32-out GEMM epilogue straight from the accumulators [1] (0: through
     * an LDS image; the same values) */
    int direct_epilogue;
    /* layers with K <= narrow_kmax [128] take the 64-wide N tile */
    int narrow_kmax;
    /* fp32 1x1 layers with Cout <= 16 (RPN / mask / box predictors) on
     * k_head_f32 [1] */
    int head_f32;
    /* fp16 1x1 stride-1 layers (Cin in {64,128,256}, Cout % 64 == 0) on the
     * streaming kernel: 0 never, 1 for M >= stream1x1_min_m [65536] (K = 256
     * only when Cout == 64) [1], 2 every eligible layer */
    int stream1x1, stream1x1_min_m;
    /* model handles: fp32 stem with the pixel normalisation folded into its
     * weights (2-channel s2d input) [1]; bottleneck conv3 + projection
     * shortcut as one GEMM: 0 off, 1 fp32 handles [1], 2 all */
    int stem_fold, fuse_shortcut;
    /* RPN top-k: every (image, level) split over several workgroups [1] */
    int rpn_sliced;
    /* ROIAlign kernel: 0 the per-sample kernel, 1 / 2 / 3 one workgroup per
     * ROI with 1 / 2 / 4 items per thread, 4 the separable form (per-bin row /
     * column weight sums) [4], 5 its row-shared form, 6 the separable form
     * with each ROI's sample window staged in LDS for >= 1024 ROIs (7: for
     * any count); XCD-contiguous ROI ranges [1]; ROIs permuted by level and
     * map band before pooling (mdx_roi_align_ex) [1] */
    int roi_mode, roi_xcd_order, roi_sorted;
    /* fp16 layers the 256x256 tile takes (large_tiles): 1 on the ping-pong
     * kernel (two wave groups one barrier apart) [1], 0 on k_convg */
    int f16_pingpong;
} mdx_policy;
int mdx_policy_defaults(mdx_policy *out);
int mdx_policy_get(mdx_policy *out);
int mdx_policy_set(const mdx_policy *policy);

/* Implicit-GEMM convolution / linear layer on MFMA:
 * out = act(conv(x, w) + bias (+ residual)).  x (N,H,W,Cin); w packed
 * [Cout][KH][KW][Cin] (FrozenBN folded); bias float32 [Cout] or NULL;
 * residual like out or NULL; relu 0/1.  out_mode 0: (N,OH,OW,Cout);
 * out_mode 1: ConvTranspose2d(k=2,s=2) pixel shuffle of a 1x1 GEMM with
 * Cout = 4*Co -> (N,2H,2W,Co).  Cin must be a multiple of 8 (fp16) / 4 (fp32). */
int mdx_conv2d(const void *x, int N, int H, int W, int Cin, const void *w, const float *bias, int Cout,
               int KH, int KW, int stride, int pad, const void *residual, int relu, int out_mode,
               int in_dtype, int out_dtype, void *out, mdx_stream_t stream);
/* mdx_conv2d with split-K: ksplit K slices write fp32 partials into workspace
 * (ksplit*M*Cout*4 bytes), a second launch sums them in fixed order and applies
 * bias/residual/ReLU.  ksplit 0 = choose from the grid size and workspace_bytes
 * (falls back to 1 slice when it does not pay or does not fit). */
/* Winograd F(m x m, 3x3), m = 2, 4 or 6, for fp32 3x3 / stride-1 / pad-1
 * convolutions (NHWC): the algorithm the model handle uses for such layers
 * with Cin >= 64 (cuDNN's WINOGRAD family, which PyTorch selects for fp32
 * 3x3 convs).  weights: w float32 OIHW [Cout][Cin][3][3] -> U float32
 * [(m+2)^2][Cout][Cin] (host function).  conv: x float32 (N,H,W,Cin), U as
 * above, bias [Cout] or NULL, optional ReLU -> out (N,H,W,Cout); workspace
 * (16-B aligned) >= mdx_winograd_workspace_bytes.  Cin % 4 == 0, Cout % 8 == 0.
 * winograd_tile: the m a policy (mdx_policy.winograd) runs an H x W layer with
 * (policy 6: 6 where the 8x8 tiles execute under 0.9x the tile products of
 * F(4,3)'s 6x6, else 4). */
int mdx_winograd_weights(const float *w, int Cout, int Cin, int m, float *U);
int64_t mdx_winograd_workspace_bytes(int N, int H, int W, int Cin, int Cout, int m);
int mdx_conv3x3_winograd(const float *x, int N, int H, int W, int Cin, const float *U, const float *bias, int Cout,
                         int relu, int m, float *out, void *workspace, int64_t workspace_bytes, mdx_stream_t stream);
/* Split-plane mode (mdx_policy.fp32_split = 6): the same layer with U also
 * split once into bf16 planes (mdx_split_x6 of U as NB*Cout rows of Cin):
 * the input transform writes V as planes and the NB GEMMs run on the 256x256
 * LDS-DMA plane kernel (k_gemm_x6); outside split mode, or with Cin % 16 != 0,
 * as mdx_conv3x3_winograd.  Model handles use it only with MDX_WINO_X6 set in
 * the environment (4 % slower end to end than k_conv_x3 on every layer). */
int mdx_conv3x3_winograd_x6(const float *x, int N, int H, int W, int Cin, const float *U, const void *U_planes,
                            const float *bias, int Cout, int relu, int m, float *out, void *workspace,
                            int64_t workspace_bytes, mdx_stream_t stream);
int mdx_winograd_tile(int H, int W, int mode);
/* fp32 GEMM on the bf16 matrix cores over operands split once into bf16
 * planes (replaces the fp32 Linear layers of Detectron2's FastRCNNConvFCHead,
 * M/model/config.py:21-94 box head, when the model handle's x6 mode is on).
 * split_x6: x float32 [rows][ldx] (first K columns, K % 16 == 0) -> planes
 * (mdx_x6_plane_bytes(rows, K) bytes): per row K/16 groups of 96 B = hi, mid,
 * lo bf16 of 16 values, x = hi + mid + lo exactly.  gemm_x6: out[m][n] =
 * act(sum_k A[m][k] B[n][k] + bias[n] (+ residual[m][n])) for A [M][K], B
 * [N][K] in plane layout, fp32 out [M][N]; six of the nine plane products
 * (the dropped ones are below one fp32 rounding of each product), fp32
 * accumulation. */
int64_t mdx_x6_plane_bytes(int64_t rows, int K);
int mdx_split_x6(const float *x, int64_t rows, int K, int64_t ldx, void *out, mdx_stream_t stream);
int mdx_gemm_x6(const void *a_planes, const void *b_planes, const float *bias, int M, int N, int K,
                const float *residual, int relu, float *out, mdx_stream_t stream);
/* Kernel chosen by this thread's last mdx_conv2d / mdx_conv2d_splitk call
 * (host-only; for per-kernel timing): *kernel = MDX_CONV_KERNEL_*, *ksplit =
 * K slices launched (the split-K reduction is a second launch). */
enum {
    MDX_CONV_KERNEL_REG128 = 0,
    MDX_CONV_KERNEL_REG64 = 1,
    MDX_CONV_KERNEL_DMA256 = 2,
    MDX_CONV_KERNEL_DMA128 = 3,
    MDX_CONV_KERNEL_STREAM1X1 = 4,
    MDX_CONV_KERNEL_HEAD1X1 = 5,
    MDX_CONV_KERNEL_WINOGRAD = 6,
    MDX_CONV_KERNEL_X3_128 = 7, /* fp32 as bf16 plane products (mdx_policy.fp32_split), 128-wide N tile */
    MDX_CONV_KERNEL_X3_64 = 8,
    MDX_CONV_KERNEL_X6DMA = 9,  /* fp32 GEMM over pre-split bf16 planes, 256x256 LDS-DMA (mdx_gemm_x6) */
    MDX_CONV_KERNEL_PW128 = 14, /* REG128 / REG64 on a pointwise layer (1x1 unpadded, Winograd GEMMs): */
    MDX_CONV_KERNEL_PW64 = 15,  /* per-row precomputed addresses (mdx_policy.pointwise) */
    MDX_CONV_KERNEL_DUAL128 = 16, /* mdx_conv2d_dual (conv3 + projection shortcut in one GEMM) */
    MDX_CONV_KERNEL_DUAL64 = 17,
    MDX_CONV_KERNEL_SB128 = 18, /* PW128 / PW64 on the single-LDS-stage k_conv_sb (mdx_policy.single_stage) */
    MDX_CONV_KERNEL_SB64 = 19,
    MDX_CONV_KERNEL_SBDUAL128 = 20, /* DUAL128 / DUAL64 on k_conv_sb */
    MDX_CONV_KERNEL_SBDUAL64 = 21,
    MDX_CONV_KERNEL_SBG128 = 22, /* REG128 / REG64 on the single-stage k_conv_sbg (mdx_policy.single_stage 2) */
    MDX_CONV_KERNEL_SBG64 = 23,
    /* profile records only (mdx_model_profile_read): the Winograd layers'
     * transforms; their GEMM is recorded under the kernel it ran on */
    MDX_CONV_KERNEL_PP16 = 26, /* fp16 256x256 ping-pong (mdx_policy.f16_pingpong) */
    MDX_CONV_KERNEL_WINO_IN = 12,
    MDX_CONV_KERNEL_WINO_OUT = 13
};
int mdx_conv2d_last_plan(int *kernel, int *ksplit);
int64_t mdx_conv2d_workspace_bytes(int N, int H, int W, int Cin, int Cout, int KH, int KW, int stride, int pad);
int mdx_conv2d_splitk(const void *x, int N, int H, int W, int Cin, const void *w, const float *bias, int Cout,
                      int KH, int KW, int stride, int pad, const void *residual, int relu, int out_mode,
                      int in_dtype, int out_dtype, void *out, int ksplit, void *workspace,
                      int64_t workspace_bytes, mdx_stream_t stream);
/* A ResNet bottleneck's conv3 and its projection shortcut as one GEMM
 * (Detectron2 BottleneckBlock.forward: out = relu(conv3(h) + shortcut(x)),
 * M/model/config.py:21-94 builds it): out = act(x . W[:, :Cin] +
 * x2[:, ::stride2, ::stride2] . W[:, Cin:] + bias), x (N,H,W,Cin),
 * x2 (N,H2,W2,Cin2), w [Cout][Cin + Cin2], both 1x1.  Cin and Cin2 multiples
 * of 32 (fp32) / 64 (fp16); dtype 0 f32, 1 f16 (in = out). */
int mdx_conv2d_dual(const void *x, int N, int H, int W, int Cin, const void *x2, int H2, int W2, int Cin2,
                    int stride2, const void *w, const float *bias, int Cout, int relu, int dtype, void *out,
                    void *workspace, int64_t workspace_bytes, mdx_stream_t stream);

/* scale_raw_frames LUT + replicate 1->C channels + (x - mean[c]) / std[c] + zero
 * pad to (Hp, Wp) with Cp (>= C) channels.  frames uint8 (B,h,w). */
int mdx_preprocess(const uint8_t *frames, int B, int h, int w, const uint8_t lut[256], const float *mean,
                   const float *std_, int C, int Cp, int Hp, int Wp, int dtype, void *out,
                   mdx_stream_t stream);

/* Same preprocessing written space-to-depth for the stride-2 stem:
 * out (B, Hp/2+1, Wp/2+1, 16): S2D pixel (Y, X) channel (2*dy+dx)*4 + c holds
 * padded pixel (2Y-1+dy, 2X-1+dx) channel c (c < C <= 4; other slots 0).
 * The 7x7/s2/p3 stem equals a 4x4/s1/p1 conv over it with weights
 * W'[o][ty][tx][(2dy+dx)*4+c] = W[o][c][2ty+dy][2tx+dx] (0 where 2ty+dy = 7). */
int mdx_preprocess_s2d(const uint8_t *frames, int B, int h, int w, const uint8_t lut[256], const float *mean,
                       const float *stdv, int C, int Hp, int Wp, int dtype, void *out, mdx_stream_t stream);
/* Same input in the 2-channel form of a stem with the normalisation folded
 * into its weights: out (B, Hp/2+1, Wp/2+1, 8) = per 2x2 phase (scaled pixel,
 * inside the image ? 1 : 0), zeros outside.  Used by fp32 model handles. */
int mdx_preprocess_s2d_folded(const uint8_t *frames, int B, int h, int w, const uint8_t lut[256], int Hp, int Wp,
                              int dtype, void *out, mdx_stream_t stream);

/* y = x converted between float32 (0) and float16 (1), round to nearest
 * even; n (elements) a multiple of 8. */
int mdx_convert(const void *x, int64_t n, int in_dtype, void *out, int out_dtype, mdx_stream_t stream);

/* max_pool2d(k, s, p), NHWC. */
int mdx_maxpool2d(const void *x, int N, int H, int W, int C, int k, int s, int p, int dtype, void *out,
                  mdx_stream_t stream);

/* GroupNorm(G, C, eps) with affine; fuse 1: out = gn + up2(up), 2: (gn + up2(up)) / 2
 * (FPN top-down, nearest x2).  workspace: >= mdx_groupnorm_workspace_bytes(N, H, W, G)
 * bytes (Welford partials + per-group mean/rstd).  C/G must be a multiple of 8. */
int64_t mdx_groupnorm_workspace_bytes(int N, int H, int W, int G);
int mdx_groupnorm(const void *x, int N, int H, int W, int C, int G, float eps, const float *gamma,
                  const float *beta, const void *up, int fuse, int dtype, void *out, float *workspace,
                  mdx_stream_t stream);


/* RPN find_top_rpn_proposals: per level head tensor float32 (B,H_l,W_l,A*5)
 * = [objectness(A), deltas(A*4)]; cell_anchors float32 [L][A][4].
 * out_boxes (B,post_topk,4), out_scores (B,post_topk) (logits, -inf pad),
 * out_count (B).  A in 1..8.  reg_weights: RPN.BBOX_REG_WEIGHTS (wx, wy, ww, wh)
 * of Box2BoxTransform, NULL = (1, 1, 1, 1).
 * workspace >= mdx_rpn_workspace_bytes(B, L, pre_topk). */
int64_t mdx_rpn_workspace_bytes(int B, int L, int pre_topk);
int mdx_rpn_proposals(const float *const *head, const int *lvl_h, const int *lvl_w, const int *strides,
                      int L, int B, int A, const float *cell_anchors, float offset, int img_h, int img_w,
                      int pre_topk, int post_topk, float nms_thresh, float min_size, float clampv,
                      const float *reg_weights, float *out_boxes, float *out_scores, int *out_count,
                      void *workspace, mdx_stream_t stream);

/* ROIPooler(ROIAlignV2): rois float32 (R,4) XYXY, R = B*per_image, rows with
 * index >= counts[b] produce zeros.  out (R,P,P,C).  dtype 0 fp32, 1 fp16
 * (features and out); 2: fp32 features, each out row of P*P*C values written
 * as bf16 planes in the mdx_split_x6 layout (mdx_x6_plane_bytes(R, P*P*C)
 * bytes; the A operand of mdx_gemm_x6), separable kernel only. */
int mdx_roi_align(const void *const *feats, const int *fh, const int *fw, const float *scales, int L,
                  int min_level, int C, const float *rois, const int *counts, int R, int per_image, int P,
                  int sampling, int aligned, float canonical_size, float canonical_level, int dtype,
                  void *out, mdx_stream_t stream);

/* Same, with an optional int32 scratch of R entries: when order_ws is not
 * NULL (and mdx_policy.roi_sorted, the default) the ROIs of each image
 * are first permuted by pyramid level and map band (k_roi_order) so the
 * workgroups in flight share one band of one level map; outputs are
 * identical to the unordered call.  order_ws == NULL is mdx_roi_align. */
int mdx_roi_align_ex(const void *const *feats, const int *fh, const int *fw, const float *scales, int L,
                     int min_level, int C, const float *rois, const int *counts, int R, int per_image, int P,
                     int sampling, int aligned, float canonical_size, float canonical_level, int dtype,
                     int *order_ws, void *out, mdx_stream_t stream);

/* fast_rcnn_inference_single_image + detector_postprocess for 1 class:
 * pred float32 (B*R, ld_pred) = [cls0, bg, dx, dy, dw, dh].  Outputs
 * (B,D,4), (B,D), int64 (B,D), ndet (B). */
int mdx_box_postprocess(const float *pred, int ld_pred, const float *proposals, const int *counts, int B,
                        int R, int D, float score_thresh, float nms_thresh, int img_h, int img_w,
                        const float *reg_weights, float clampv, float *det_boxes, float *det_scores,
                        int64_t *det_classes, int *ndet, mdx_stream_t stream);

/* mask_rcnn_inference sigmoid + paste_masks_in_image (grid_sample) >= thresh:
 * logits float32 (B*D, M, M) -> out uint8, plane r = b*D + d at
 * out + r*plane_stride (img_h x img_w, row-major; plane_stride >= img_h*img_w,
 * a multiple of 16 keeps every plane 16-B aligned). */
int mdx_paste_masks(const float *logits, const float *boxes, const int *counts, int B, int D, int M,
                    int img_h, int img_w, int64_t plane_stride, float thresh, uint8_t *out,
                    mdx_stream_t stream);

/* keypoint head score_lowres ConvTranspose2d(k=4, s=2, p=1) second half:
 * y float32 (R*Hi*Wi, Co*16) = mdx_conv2d(x, W[co*16+ky*4+kx][ci]) ->
 * out float32 (R, Co, 2Hi, 2Wi) (col2im + bias). */
int mdx_deconv_col2im(const float *y, const float *bias, int R, int Hi, int Wi, int Co, float *out,
                      mdx_stream_t stream);

/* F.interpolate(scale_factor=2, bilinear, align_corners=False), float32 NCHW. */
int mdx_upsample_bilinear2x(const float *x, int NC, int H, int W, float *out, mdx_stream_t stream);

/* ProcessFeaturesStep.__nms_mask_instances (mask-IoU NMS, reference quirks
 * kept; M/pipeline/process_features_step.py:63-113) + instance-0 selection of
 * mask_and_keypoints_from_model_output (M/proc/proc.py:657-685).
 * masks uint8 planes of plane_stride bytes (B*D planes of h*w), scores (B,D),
 * ndet (B), kpts float32 (B,D,K,3) ->
 * keep_idx int32 (B,D) (-1 padded, pick order), nkeep (B), sel_mask uint8
 * (B,h,w), sel_kpts float64 (B,K,3) (NaN when no instance). */
int mdx_mask_nms_select(const uint8_t *masks, int64_t plane_stride, const float *scores, const int *ndet,
                        const float *kpts, int B, int D, int K, int h, int w, float iou_thresh, int *keep_idx,
                        int *nkeep, uint8_t *sel_mask, double *sel_kpts, mdx_stream_t stream);

/* Centres of the kept detections for the instance tracker
 * (ProcessFeaturesStep.__instances_to_detections,
 * M/pipeline/process_features_step.py:116-130): per frame b and kept slot
 * s < nkeep[b], scipy center_of_mass (row, col) of mask plane keep_idx[b,s], or
 * the box centre (x, y) when that mask is empty.  masks/plane_stride/keep_idx/
 * nkeep as mdx_mask_nms_select, boxes float32 (B,D,4) XYXY -> centers float64
 * (B,D,2), NaN for slots >= nkeep. */
int mdx_mask_centers(const uint8_t *masks, int64_t plane_stride, const int *keep_idx, const int *nkeep,
                     const float *boxes, int B, int D, int h, int w, double *centers, mdx_stream_t stream);

/* Instance-selection fix-up (ProcessFeaturesStep.__select_instances,
 * M/pipeline/process_features_step.py:150-158, then instance 0 of
 * mask_and_keypoints_from_model_output, M/proc/proc.py:680-684): for i < n,
 * plane dst_idx[i] of dst (planes of plane_bytes) <- the plane_bytes at the
 * device address src_ptrs[i] (0 = all-zero plane, the empty-instances case).
 * src_ptrs / dst_idx are device arrays. */
int mdx_gather_planes(const uint64_t *src_ptrs, const int *dst_idx, uint8_t *dst, int64_t plane_bytes, int n,
                      mdx_stream_t stream);

/* heatmaps_to_keypoints: maps float32 (B*D, K, M, M) -> (B*D, K, 3) [x, y, score]. */
int mdx_heatmaps_to_keypoints(const float *maps, const float *boxes, const int *counts, int B, int D,
                              int K, int M, float *out, mdx_stream_t stream);

/* ---------------------------------------------------------------------
 * Model handle: the whole Mask/Keypoint R-CNN forward as one C call.
 * Replaces Predictor.from_config (M/model/predict.py:31-44: build_model +
 * DetectionCheckpointer.load) and Predictor.__call__'s model(inputs)
 * (:53-102, eval-mode GeneralizedRCNN.inference + detector_postprocess).
 * ------------------------------------------------------------------- */

/* Inference hyper-parameters of the Detectron2 CfgNode the reference builds
 * (get_base_config, M/model/config.py:21-94, add_dataset_cfg :113-150, the
 * InferenceStep overrides M/pipeline/inference_step.py:48-51).  Only these
 * architectures are supported: ResNet-50/101 (FrozenBN, num_groups 1), FPN
 * with GN, avg or sum fuse, LastLevelMaxPool, StandardRPNHead, 1+ box FCs,
 * MaskRCNNConvUpsampleHead, KRCNNConvDeconvUpsampleHead. */
typedef struct mdx_model_cfg {
    int depth;                     /* MODEL.RESNETS.DEPTH: 50 or 101 */
    int dtype;                     /* arithmetic: 0 = float32, 1 = float16 (fp32 accumulation) */
    int stem_out_channels;         /* 64 */
    int res2_out_channels;         /* 256 */
    int width_per_group;           /* 64 (NUM_GROUPS must be 1) */
    int stride_in_1x1;             /* 1 */
    int fpn_out_channels;          /* 256 */
    int fpn_fuse_avg;              /* FPN.FUSE_TYPE: 1 = "avg", 0 = "sum" */
    int gn_groups;                 /* 32 (FPN.NORM must be "GN") */
    float gn_eps;                  /* 1e-5 */
    int n_anchor_sizes;            /* 5, one per level p2..p6 */
    float anchor_sizes[5];         /* 32 64 128 256 512 */
    int n_aspect_ratios;           /* 3 (1..8, the same at every level) */
    float aspect_ratios[8];        /* 0.5 1 2 */
    float anchor_offset;           /* 0 */
    int rpn_pre_nms_topk;          /* PRE_NMS_TOPK_TEST 1000 */
    int rpn_post_nms_topk;         /* POST_NMS_TOPK_TEST 1000 */
    float rpn_nms_thresh;          /* 0.7 */
    float rpn_min_box_size;        /* 0 */
    int num_classes;               /* ROI_HEADS.NUM_CLASSES (must be 1) */
    float score_thresh;            /* SCORE_THRESH_TEST (--instance-threshold) */
    float nms_thresh;              /* NMS_THRESH_TEST 0.5 */
    int detections_per_image;      /* TEST.DETECTIONS_PER_IMAGE (--allowed-detections) */
    int box_pooler_resolution;     /* 7 */
    int box_num_fc;                /* 2 */
    int box_fc_dim;                /* 1024 */
    float box_reg_weights[4];      /* 10 10 5 5 */
    int mask_on;                   /* 1 */
    int mask_pooler_resolution;    /* 14 */
    int mask_num_conv;             /* 4 */
    int mask_conv_dim;             /* 256 */
    float mask_threshold;          /* 0.5 (paste_masks_in_image) */
    int keypoint_on;               /* 1 */
    int keypoint_pooler_resolution;/* 7 (M/model/config.py:84) */
    int n_keypoint_convs;          /* 8 */
    int keypoint_conv_dims[16];    /* 512 x 8 */
    int num_keypoints;             /* 8 */
    int pooler_sampling_ratio;     /* 0 (adaptive) */
    int pooler_aligned;            /* 1 (ROIAlignV2) */
    float canonical_box_size;      /* 224 */
    float canonical_level;         /* 4 */
    int in_channels;               /* 3 (INPUT.FORMAT RGB: the gray frame replicated) or 1 */
    float pixel_mean[3];           /* 1.12 x3 (M/model/config.py:141-148) */
    float pixel_std[3];            /* 5.79 x3 */
    int size_divisibility;         /* 32 */
    float rpn_bbox_reg_weights[4]; /* RPN.BBOX_REG_WEIGHTS 1 1 1 1 */
    int head_dtype;                /* mask + keypoint heads: 0 = dtype, 1 = float16 (with dtype 0: the
                                      fp32 trunk / RPN / box head and fp16 mask + keypoint heads of
                                      BASELINE config 5; pooled in fp32, converted) */
} mdx_model_cfg;

typedef void *mdx_model_t;


/* Weights blob: Detectron2 state-dict layout (parameter / buffer names of
 * GeneralizedRCNN, e.g. "backbone.bottom_up.res2.0.conv1.weight"), serialised
 * as  "MDXW" | u32 version (1) | u32 count | count x { u32 name_len | name |
 * u32 ndim | i64 shape[ndim] | float32 data[prod(shape)] }  (little endian).
 * Create folds FrozenBN into the convs, packs every weight once into the
 * kernels' layouts (NHWC/OHWI, fp16 when cfg->dtype == 1) and uploads them
 * to `device`; it synchronises the host.  Missing or mis-shaped tensors fail
 * with MDX_EINVAL naming the key. */
int mdx_model_create(const void *weights_blob, int64_t blob_bytes, const mdx_model_cfg *cfg, int device,
                     mdx_model_t *out);
int mdx_model_destroy(mdx_model_t model);
/* The policy this handle runs with (captured at mdx_model_create). */
int mdx_model_get_policy(mdx_model_t model, mdx_policy *out);

/* Caller-owned device outputs of one forward over B frames of h x w
 * (D = detections_per_image, K = num_keypoints, S = 4 * keypoint pooler
 * resolution).  Detections are score-ordered, rows >= ndet[b] are padding.
 * masks: B*D planes at masks + (b*D+d)*mask_plane_stride (h x w bytes,
 * 0/1), may be NULL; keypoints (B,D,K,3) [x, y, score] may be NULL;
 * keypoint_heatmaps (B,D,K,S,S) may be NULL (then kept in the workspace). */
typedef struct mdx_model_outputs {
    float *boxes;               /* (B,D,4) XYXY, image pixels */
    float *scores;              /* (B,D) */
    int64_t *classes;           /* (B,D) */
    int32_t *ndet;              /* (B) */
    uint8_t *masks;
    int64_t mask_plane_stride;  /* >= h*w; a multiple of 16 keeps planes 16-B aligned */
    float *keypoints;
    float *keypoint_heatmaps;
} mdx_model_outputs;

/* Reserve the workspace for forwards of up to B frames of h x w on `stream`
 * (each stream has its own workspace, so forwards on different streams may
 * run concurrently).  Allocates (device memory, synchronous): call it before
 * capturing forwards into a HIP graph.  mdx_model_forward reserves on demand. */
int mdx_model_reserve(mdx_model_t model, int B, int h, int w, mdx_stream_t stream);

/* One forward: frames uint8 (B,h,w) device (the gray depth frame; replicated
 * to in_channels as Predictor.__call__ does, M/model/predict.py:74-77); lut
 * host uint8[256] applied first (scale_raw_frames fused; NULL = identity).
 * Everything is enqueued on `stream` with no host synchronisation (fixed
 * shapes: rpn_post_nms_topk proposals and D detections per image, counts on
 * the device), so the call can be captured into a HIP graph once reserved. */
int mdx_model_forward(mdx_model_t model, const uint8_t *frames, int B, int h, int w, const uint8_t *lut,
                      const mdx_model_outputs *out, mdx_stream_t stream);

/* Intermediates of the last forward on `stream` (valid until the next forward
 * on it), for stage-wise parity tests: "input" (B,Hp,Wp,4 NHWC), "res2".."res5",
 * "p2".."p6" (NHWC), per FPN level l "fpn_lateral<l>" (lateral conv),
 * "fpn_inner<l>" (its GroupNorm + top-down fuse), "fpn_output<l>" (output conv
 * before GroupNorm), "proposals" (B,P,4) f32, "proposal_scores" (B,P) f32,
 * "proposal_count" (B) i32, "box_pooled" (B*P,R,R,C), "box_pred" (B*P,6) f32,
 * "mask_logits" (B*D,2M,2M,1) f32.  shape[4] gets the dims (unused = 1),
 * dtype: 0 f32, 1 f16, 2 i32.  copy: D2D copy of `bytes` into dst on `stream`. */
int mdx_model_tensor_info(mdx_model_t model, mdx_stream_t stream, const char *name, int64_t shape[4], int *dtype);
int mdx_model_tensor_copy(mdx_model_t model, mdx_stream_t stream, const char *name, void *dst, int64_t bytes);

/* Testing aid: reserve the workspace of `stream` for (B, h, w) and fill all of
 * it with `byte` (asynchronously on `stream`), so a test can show that a
 * forward's results do not depend on what the workspace held before. */
int mdx_model_debug_fill(mdx_model_t model, int B, int h, int w, int byte, mdx_stream_t stream);

/* Testing aid: the byte size of `stream`'s workspace, the offset of a named
 * intermediate in it (-1 when it lives in a caller buffer), and a D2D copy of
 * its first dst_bytes bytes into dst (each part skipped when its pointer is
 * NULL). */
int mdx_model_debug_arena(mdx_model_t model, mdx_stream_t stream, const char *name, int64_t *offset,
                          int64_t *arena_bytes, void *dst, int64_t dst_bytes);

/* Per-convolution timing of later forwards (HIP events around every conv
 * launch; host-only bookkeeping, off by default).  read: after the stream
 * is synchronised, up to max records {kernel (MDX_CONV_KERNEL_*), ksplit, M,
 * N, K, algorithmic FLOP, milliseconds} of the last profiled forward; returns
 * the number written.  A Winograd layer gives three records: its input
 * transform (MDX_CONV_KERNEL_WINO_IN; M = tiles, N = Cin, K = (m+2)^2, flop =
 * the transform's algorithmic HBM bytes), the batched GEMM under the kernel
 * that ran it (M = (m+2)^2 * tiles, N = Cout, K = Cin, flop = its executed
 * FLOP) and the output transform (MDX_CONV_KERNEL_WINO_OUT, bytes as for the
 * input). */
typedef struct mdx_conv_record {
    int kernel, ksplit;
    int64_t M, N, K;
    double flop, ms;
    int dtype;  /* the MFMA operand type of the launch: 0 f32, 1 f16 (config 5 mixes them) */
    int reserved;
} mdx_conv_record;
int mdx_model_profile(mdx_model_t model, int on);
int mdx_model_profile_read(mdx_model_t model, mdx_conv_record *out, int max);

#ifdef __cplusplus
}
#endif
#endif /* MDX_H_ */
