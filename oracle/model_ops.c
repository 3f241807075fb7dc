// C restatement of the two torchvision CPU kernels on the model path whose
// pure-torch restatement (model_ref.roi_align / model_ref.nms) is far too slow
// for full-size frames.  TEST INFRASTRUCTURE ONLY (checker + cpu_baseline).
//
// torchvision is not in this image and unpinned in the reference
// (README.md:16, setup.py:25-48); these follow its published CPU kernels:
//   roi_align_forward_kernel_impl (ops/cpu/roi_align_kernel.cpp): per ROI a
//     pre-calculated table of (4 positions, 4 bilinear weights) per
//     (ph, pw, iy, ix) sample, then per channel the sample sum in that order,
//     divided by count = max(grid_h * grid_w, 1);
//   nms_kernel_impl (ops/cpu/nms_kernel.cpp): greedy suppression over the
//     score order with IoU = inter / (area_i + area_j - inter) > threshold.
// Both are float32 with every rounding step as written (built with
// -ffp-contract=off), so they equal model_ref's torch restatements bit for bit
// (tests/test_oracle_model_ops.py).  ROIs run in parallel (OpenMP), each ROI's
// arithmetic is sequential, so the thread count does not change the result.
#include <math.h>
#include <stdint.h>
#include <stdlib.h>

typedef struct {
    int64_t p1, p2, p3, p4;
    float w1, w2, w3, w4;
} PreCalc;

static void pre_calc_roi(int H, int W, int P, int gh, int gw, float sh, float sw, float bh, float bw, PreCalc *pc) {
    int k = 0;
    for (int ph = 0; ph < P; ++ph)
        for (int pw = 0; pw < P; ++pw)
            for (int iy = 0; iy < gh; ++iy) {
                const float yy = sh + (float)ph * bh + (float)(iy + .5f) * bh / (float)gh;
                for (int ix = 0; ix < gw; ++ix) {
                    const float xx = sw + (float)pw * bw + (float)(ix + .5f) * bw / (float)gw;
                    PreCalc *c = &pc[k++];
                    float y = yy, x = xx;
                    if (y < -1.0 || y > H || x < -1.0 || x > W) {
                        c->p1 = c->p2 = c->p3 = c->p4 = 0;
                        c->w1 = c->w2 = c->w3 = c->w4 = 0.f;
                        continue;
                    }
                    if (y <= 0) y = 0;
                    if (x <= 0) x = 0;
                    int yl = (int)y, xl = (int)x, yh, xh;
                    if (yl >= H - 1) {
                        yh = yl = H - 1;
                        y = (float)yl;
                    } else {
                        yh = yl + 1;
                    }
                    if (xl >= W - 1) {
                        xh = xl = W - 1;
                        x = (float)xl;
                    } else {
                        xh = xl + 1;
                    }
                    const float ly = y - yl, lx = x - xl;
                    const float hy = (float)(1. - ly), hx = (float)(1. - lx);
                    c->p1 = (int64_t)yl * W + xl;
                    c->p2 = (int64_t)yl * W + xh;
                    c->p3 = (int64_t)yh * W + xl;
                    c->p4 = (int64_t)yh * W + xh;
                    c->w1 = hy * hx;
                    c->w2 = hy * lx;
                    c->w3 = ly * hx;
                    c->w4 = ly * lx;
                }
            }
}

// feat (N, C, H, W) f32; rois (R, 5) f32 = (batch, x1, y1, x2, y2);
// out (R, C, P, P) f32
void orc_roi_align(const float *feat, int N, int C, int H, int W, const float *rois, int R, int P, float scale,
                   int sampling, int aligned, float *out) {
    (void)N;
#pragma omp parallel for schedule(dynamic, 4)
    for (int r = 0; r < R; ++r) {
        const float *roi = rois + (int64_t)r * 5;
        const int b = (int)roi[0];
        const float off = aligned ? 0.5f : 0.f;
        const float sw = roi[1] * scale - off, sh = roi[2] * scale - off;
        const float ew = roi[3] * scale - off, eh = roi[4] * scale - off;
        float rw = ew - sw, rh = eh - sh;
        if (!aligned) {
            rw = rw > 1.f ? rw : 1.f;
            rh = rh > 1.f ? rh : 1.f;
        }
        const float bh = rh / (float)P, bw = rw / (float)P;
        const int gh = sampling > 0 ? sampling : (int)ceilf(rh / (float)P);
        const int gw = sampling > 0 ? sampling : (int)ceilf(rw / (float)P);
        const float count = (float)(gh * gw > 1 ? gh * gw : 1);
        const int ns = gh * gw;
        PreCalc *pc = (PreCalc *)malloc(sizeof(PreCalc) * (size_t)(P * P * (ns > 0 ? ns : 1)));
        pre_calc_roi(H, W, P, gh, gw, sh, sw, bh, bw, pc);
        for (int c = 0; c < C; ++c) {
            const float *d = feat + ((int64_t)b * C + c) * H * W;
            float *o = out + ((int64_t)r * C + c) * P * P;
            int k = 0;
            for (int q = 0; q < P * P; ++q) {
                float v = 0.f;
                for (int s = 0; s < ns; ++s, ++k) {
                    const PreCalc *e = &pc[k];
                    v += e->w1 * d[e->p1] + e->w2 * d[e->p2] + e->w3 * d[e->p3] + e->w4 * d[e->p4];
                }
                o[q] = v / count;
            }
        }
        free(pc);
    }
}

// boxes (n, 4) f32 x1 y1 x2 y2; order: indices by descending score (stable);
// keep receives the kept indices in order; returns their count
int orc_nms(const float *boxes, const int64_t *order, int n, float thresh, int64_t *keep) {
    float *area = (float *)malloc(sizeof(float) * (size_t)(n > 0 ? n : 1));
    unsigned char *sup = (unsigned char *)calloc((size_t)(n > 0 ? n : 1), 1);
    for (int i = 0; i < n; ++i) area[i] = (boxes[4 * i + 2] - boxes[4 * i]) * (boxes[4 * i + 3] - boxes[4 * i + 1]);
    int nk = 0;
    for (int a = 0; a < n; ++a) {
        const int64_t i = order[a];
        if (sup[i]) continue;
        keep[nk++] = i;
        const float ix1 = boxes[4 * i], iy1 = boxes[4 * i + 1], ix2 = boxes[4 * i + 2], iy2 = boxes[4 * i + 3];
        const float ia = area[i];
        for (int b = a + 1; b < n; ++b) {
            const int64_t j = order[b];
            if (sup[j]) continue;
            const float xx1 = ix1 > boxes[4 * j] ? ix1 : boxes[4 * j];
            const float yy1 = iy1 > boxes[4 * j + 1] ? iy1 : boxes[4 * j + 1];
            const float xx2 = ix2 < boxes[4 * j + 2] ? ix2 : boxes[4 * j + 2];
            const float yy2 = iy2 < boxes[4 * j + 3] ? iy2 : boxes[4 * j + 3];
            const float w = xx2 - xx1 > 0.f ? xx2 - xx1 : 0.f;
            const float h = yy2 - yy1 > 0.f ? yy2 - yy1 : 0.f;
            const float inter = w * h;
            const float ovr = inter / (ia + area[j] - inter);
            if (ovr > thresh) sup[j] = 1;
        }
    }
    free(area);
    free(sup);
    return nk;
}
