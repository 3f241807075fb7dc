/*
 * oracle/frameops.c -- CPU restatement of the reference frame ops.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product path links, loads or
 * calls this file: it is the parity checker used by tests/, by
 * __graft_entry__.smoke() and by bench.py's cpu_baseline leg.
 *
 * Every function restates the reference (moseq2_detectron_extract, "M/")
 * together with the third-party semantics it relies on.  OpenCV is NOT in
 * this image, so the OpenCV-backed parts are restated from OpenCV 4.x's
 * published algorithms (see DESIGN.md "Oracle"):
 *
 *   orc_prep            M/proc/proc.py:129-172 prep_raw_frames (numpy part),
 *                       :175-186 find_invalid_pixels, M/proc/roi.py:215-254
 *                       apply_roi/get_bbox.  PINNED by tests/golden fixtures
 *                       generated from the reference itself.
 *   orc_scale_lut       M/proc/proc.py:214-234 scale_raw_frames.  PINNED.
 *   orc_inpaint_ns      M/proc/proc.py:189-210 -> cv2.inpaint(..,3,INPAINT_NS)
 *                       (OpenCV imgproc/inpaint.cpp icvNSInpaintFMM, restated;
 *                       parity unpinned)
 *   orc_median3         M/proc/proc.py:506 cv2.medianBlur(f, 3), BORDER_REPLICATE
 *   orc_morph           M/proc/proc.py:509 cv2.morphologyEx(MORPH_OPEN, ellipse9,
 *                       iterations) = erode^it then dilate^it, default border
 *                       (+inf for erode, -inf for dilate)
 *   orc_frame_features  M/proc/proc.py:237-302 get_frame_features + :518-549
 *                       im_moment_features: Suzuki85 outer border of each
 *                       8-connected blob, contourArea, polygon cv2.moments
 *   orc_crop_rotate     M/proc/proc.py:305-340 crop_and_rotate_frame:
 *                       copyMakeBorder + getRotationMatrix2D + warpAffine
 *                       (INTER_LINEAR fixed-point path, AB_BITS=10, INTER_BITS=5)
 *
 * Build: oracle/Makefile  (gcc -O2 -ffp-contract=off: no FMA contraction so
 * the double/float rounding sequence is the one written here).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <float.h>

/* ------------------------------------------------------------------ */
/* prep_raw_frames (numpy part) + find_invalid_pixels + apply_roi      */
/* ------------------------------------------------------------------ */
/* numpy float64 -> uint8 astype on x86: truncation toward zero through a
 * 32-bit integer conversion (values are within [vmin, vmax] here). */
static inline uint8_t f64_to_u8_numpy(double v) { return (uint8_t)(int32_t)v; }

void orc_prep(const int16_t *raw, int64_t n, int H, int W, const double *bg,
              const uint8_t *roi, int y0, int y1, int x0, int x1,
              int has_vmin, double vmin, int has_vmax, double vmax,
              uint8_t *out, uint8_t *invalid)
{
    const int oh = y1 - y0, ow = x1 - x0;
    for (int64_t f = 0; f < n; ++f) {
        const int16_t *src = raw + f * (int64_t)H * W;
        for (int y = 0; y < oh; ++y) {
            for (int x = 0; x < ow; ++x) {
                const int64_t si = (int64_t)(y + y0) * W + (x + x0);
                const int16_t r = src[si];
                /* bground_im - frames, float64 (int16 promotes exactly) */
                double v = bg ? bg[si] - (double)r : (double)r;
                if (roi) v = v * (double)roi[si];
                if (has_vmin && v < vmin) v = 0.0;
                if (has_vmax && v > vmax) v = vmax;
                const int64_t oi = f * (int64_t)oh * ow + (int64_t)y * ow + x;
                out[oi] = f64_to_u8_numpy(v);
                if (invalid) invalid[oi] = (uint8_t)((r == 0) * (roi ? roi[si] : 1));
            }
        }
    }
}

/* scale_raw_frames(frames, vmin, vmax, 'uint8') as a 256-entry table:
 * ((x - vmin) * ((255 - 0) / (vmax - vmin)) + 0).astype(uint8), float64.
 * int_vmin: vmin is a Python int, so numpy evaluates uint8 - vmin in uint8
 * (wraps modulo 256) before promoting to float64 (pinned by the golden). */
void orc_scale_lut(double vmin, double vmax, int int_vmin, uint8_t *lut)
{
    const double k = (255.0 - 0.0) / (vmax - vmin);
    for (int v = 0; v < 256; ++v) {
        const double d = int_vmin ? (double)(uint8_t)(v - (int)vmin) : (double)v - vmin;
        lut[v] = f64_to_u8_numpy(d * k + 0.0);
    }
}

/* ------------------------------------------------------------------ */
/* cv2.medianBlur(ksize=3), BORDER_REPLICATE                           */
/* ------------------------------------------------------------------ */
#define SORT2(a, b) do { if (a > b) { uint8_t t_ = a; a = b; b = t_; } } while (0)
/* median of 9 by a fixed compare-exchange network (the middle order statistic) */
static inline uint8_t median9(uint8_t p0, uint8_t p1, uint8_t p2, uint8_t p3, uint8_t p4, uint8_t p5,
                              uint8_t p6, uint8_t p7, uint8_t p8)
{
    SORT2(p1, p2); SORT2(p4, p5); SORT2(p7, p8); SORT2(p0, p1); SORT2(p3, p4); SORT2(p6, p7);
    SORT2(p1, p2); SORT2(p4, p5); SORT2(p7, p8); SORT2(p0, p3); SORT2(p5, p8); SORT2(p4, p7);
    SORT2(p3, p6); SORT2(p1, p4); SORT2(p2, p5); SORT2(p4, p7); SORT2(p4, p2); SORT2(p6, p4);
    SORT2(p4, p2);
    return p4;
}

void orc_median3(const uint8_t *src, int64_t n, int H, int W, uint8_t *dst)
{
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t f = 0; f < n; ++f) {
        const uint8_t *s = src + f * (int64_t)H * W;
        uint8_t *d = dst + f * (int64_t)H * W;
        for (int y = 0; y < H; ++y) {
            const uint8_t *r0 = s + (int64_t)(y > 0 ? y - 1 : 0) * W, *r1 = s + (int64_t)y * W;
            const uint8_t *r2 = s + (int64_t)(y < H - 1 ? y + 1 : H - 1) * W;
            for (int x = 0; x < W; ++x) {
                const int xl = x > 0 ? x - 1 : 0, xr = x < W - 1 ? x + 1 : W - 1;
                d[(int64_t)y * W + x] = median9(r0[xl], r0[x], r0[xr], r1[xl], r1[x], r1[xr], r2[xl], r2[x], r2[xr]);
            }
        }
    }
}

/* ------------------------------------------------------------------ */
/* erode / dilate with an arbitrary structuring element, OpenCV default */
/* border (pixels outside the image never win the min / max).          */
/* ------------------------------------------------------------------ */
static void morph_once(const uint8_t *s, uint8_t *d, int H, int W,
                       const uint8_t *strel, int kh, int kw, int is_dilate, uint8_t *rows)
{
    const int ay = kh / 2, ax = kw / 2;  /* default anchor = centre */
    /* each strel row as one run [k0, k1] when it is contiguous: the min / max
     * over the element is the min / max over its rows of the horizontal run
     * extremum (clipped to the image, i.e. outside pixels ignored) */
    int k0[32], k1[32], runs = kh <= 32;
    for (int ky = 0; ky < kh && runs; ++ky) {
        k0[ky] = -1; k1[ky] = -2;
        for (int kx = 0; kx < kw; ++kx)
            if (strel[ky * kw + kx]) { if (k0[ky] < 0) k0[ky] = kx; k1[ky] = kx; }
        for (int kx = k0[ky] < 0 ? kw : k0[ky]; kx <= k1[ky]; ++kx)
            if (!strel[ky * kw + kx]) runs = 0;
    }
    if (runs && rows) {
        /* rows[slot][y][x] = horizontal extremum of row y over a distinct run
         * (strel rows with the same run share a slot) */
        int slot[32];
        for (int ky = 0; ky < kh; ++ky) {
            slot[ky] = ky;
            for (int j = 0; j < ky; ++j)
                if (k0[j] == k0[ky] && k1[j] == k1[ky]) { slot[ky] = slot[j]; break; }
        }
        for (int ky = 0; ky < kh; ++ky) {
            if (k0[ky] < 0 || slot[ky] != ky) continue;
            uint8_t *o = rows + (int64_t)ky * H * W;
            for (int y = 0; y < H; ++y) {
                const uint8_t *r = s + (int64_t)y * W;
                for (int x = 0; x < W; ++x) {
                    int a = x + k0[ky] - ax, b = x + k1[ky] - ax;
                    a = a < 0 ? 0 : a; b = b >= W ? W - 1 : b;
                    int acc = is_dilate ? 0 : 255;
                    for (int xx = a; xx <= b; ++xx) {
                        const int v = r[xx];
                        if (is_dilate) { if (v > acc) acc = v; } else { if (v < acc) acc = v; }
                    }
                    o[(int64_t)y * W + x] = (uint8_t)acc;
                }
            }
        }
        for (int y = 0; y < H; ++y)
            for (int x = 0; x < W; ++x) {
                int acc = is_dilate ? 0 : 255;
                for (int ky = 0; ky < kh; ++ky) {
                    const int yy = y + ky - ay;
                    if (k0[ky] < 0 || yy < 0 || yy >= H) continue;
                    const int v = rows[((int64_t)slot[ky] * H + yy) * W + x];
                    if (is_dilate) { if (v > acc) acc = v; } else { if (v < acc) acc = v; }
                }
                d[(int64_t)y * W + x] = (uint8_t)acc;
            }
        return;
    }
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x) {
            int acc = is_dilate ? 0 : 255;
            for (int ky = 0; ky < kh; ++ky)
                for (int kx = 0; kx < kw; ++kx) {
                    if (!strel[ky * kw + kx]) continue;
                    const int yy = y + ky - ay, xx = x + kx - ax;
                    if (yy < 0 || yy >= H || xx < 0 || xx >= W) continue;
                    const int v = s[yy * W + xx];
                    if (is_dilate) { if (v > acc) acc = v; }
                    else { if (v < acc) acc = v; }
                }
            d[y * W + x] = (uint8_t)acc;
        }
}

/* op: 0 erode, 1 dilate, 2 open (erode^it, dilate^it), 3 close */
void orc_morph(const uint8_t *src, int64_t n, int H, int W, int op,
               const uint8_t *strel, int kh, int kw, int iters, uint8_t *dst)
{
#pragma omp parallel for schedule(dynamic, 1)
    for (int64_t f = 0; f < n; ++f) {
        uint8_t *a = (uint8_t *)malloc((size_t)H * W), *b = (uint8_t *)malloc((size_t)H * W);
        uint8_t *rows = kh <= 32 ? (uint8_t *)malloc((size_t)kh * H * W) : NULL;
        memcpy(a, src + f * (int64_t)H * W, (size_t)H * W);
        int passes[2] = {0, 0}, nph = 1;
        if (op == 0) passes[0] = 0;
        else if (op == 1) passes[0] = 1;
        else if (op == 2) { passes[0] = 0; passes[1] = 1; nph = 2; }
        else { passes[0] = 1; passes[1] = 0; nph = 2; }
        for (int p = 0; p < nph; ++p)
            for (int it = 0; it < iters; ++it) {
                morph_once(a, b, H, W, strel, kh, kw, passes[p], rows);
                uint8_t *t = a; a = b; b = t;
            }
        memcpy(dst + f * (int64_t)H * W, a, (size_t)H * W);
        free(a); free(b); free(rows);
    }
}

/* ------------------------------------------------------------------ */
/* findContours(RETR_TREE, CHAIN_APPROX_SIMPLE) + contourArea argmax +  */
/* cv2.moments(contour) + im_moment_features                            */
/* ------------------------------------------------------------------ */
/* Chain-code deltas, OpenCV order: 0=E,1=NE,2=N,3=NW,4=W,5=SW,6=S,7=SE
 * (image coordinates, y grows downwards). */
static const int CDX[8] = {1, 1, 0, -1, -1, -1, 0, 1};
static const int CDY[8] = {0, -1, -1, -1, 0, 1, 1, 1};

typedef struct { int64_t a00, a10, a01, a20, a11, a02; } green_t;

/* Green's-theorem sums of cv::contourMoments for one closed polygon edge
 * (x1,y1)->(x2,y2).  All quantities are integers, so int64 sums are exact and
 * equal OpenCV's double sums (which are exact below 2^53 at these sizes). */
static inline void green_edge(green_t *g, int64_t xi_1, int64_t yi_1, int64_t xi, int64_t yi)
{
    const int64_t xi2 = xi * xi, yi2 = yi * yi;
    const int64_t dxy = xi_1 * yi - xi * yi_1;
    const int64_t xii_1 = xi_1 + xi, yii_1 = yi_1 + yi;
    g->a00 += dxy;
    g->a10 += dxy * xii_1;
    g->a01 += dxy * yii_1;
    g->a20 += dxy * (xi_1 * xii_1 + xi2);
    g->a11 += dxy * (xi_1 * (yii_1 + yi_1) + xi * (yii_1 + yi));
    g->a02 += dxy * (yi_1 * yii_1 + yi2);
}

/* Follow the outer border starting at fg pixel (x0,y0) whose west neighbour
 * is background (Suzuki & Abe 1985, as coded in OpenCV icvFetchContour).
 * img: padded binary image (1-pixel zero frame), stride PW, coordinates are
 * padded; emitted vertices are un-padded (x-1, y-1). */
static green_t trace_outer(const uint8_t *img, int PW, int x0, int y0)
{
    green_t g = {0, 0, 0, 0, 0, 0};
    int s = 4, s_end = 4;
    int x1 = 0, y1 = 0;
    /* clockwise search from the west neighbour */
    do {
        s = (s - 1) & 7;
        x1 = x0 + CDX[s]; y1 = y0 + CDY[s];
    } while (img[y1 * PW + x1] == 0 && s != s_end);
    if (s == s_end) return g; /* isolated pixel: single-point contour */
    int x3 = x0, y3 = y0;
    int px = x0 - 1, py = y0 - 1; /* previous emitted vertex (un-padded) */
    const int sx = px, sy = py;
    int first = 1;
    for (;;) {
        /* counter-clockwise search around (x3,y3) starting after s */
        int x4 = 0, y4 = 0;
        for (int c = 0; c < 8; ++c) {
            s = (s + 1) & 7;
            x4 = x3 + CDX[s]; y4 = y3 + CDY[s];
            if (img[y4 * PW + x4]) break;
        }
        if (!first) { green_edge(&g, px, py, x3 - 1, y3 - 1); px = x3 - 1; py = y3 - 1; }
        first = 0;
        if (x4 == x0 && y4 == y0 && x3 == x1 && y3 == y1) break;
        x3 = x4; y3 = y4;
        s = (s + 4) & 7;
    }
    /* close the polygon back to the start vertex */
    green_edge(&g, px, py, sx, sy);
    return g;
}

/* OpenCV contourMoments scaling + completeMomentState, then
 * im_moment_features (numpy float64). */
static void moments_to_features(const green_t *g, double *cx, double *cy,
                                double *orient, double *ax0, double *ax1)
{
    const double nan = NAN;
    double m00 = 0, m10 = 0, m01 = 0, m20 = 0, m11 = 0, m02 = 0;
    const double a00 = (double)g->a00;
    if (fabs(a00) > FLT_EPSILON) {
        double db1_2, db1_6, db1_12, db1_24;
        if (a00 > 0) {
            db1_2 = 0.5; db1_6 = 0.16666666666666666666666666666667;
            db1_12 = 0.083333333333333333333333333333333; db1_24 = 0.041666666666666666666666666666667;
        } else {
            db1_2 = -0.5; db1_6 = -0.16666666666666666666666666666667;
            db1_12 = -0.083333333333333333333333333333333; db1_24 = -0.041666666666666666666666666666667;
        }
        m00 = a00 * db1_2;
        m10 = (double)g->a10 * db1_6;
        m01 = (double)g->a01 * db1_6;
        m20 = (double)g->a20 * db1_12;
        m11 = (double)g->a11 * db1_24;
        m02 = (double)g->a02 * db1_12;
    }
    double mcx = 0, mcy = 0;
    if (fabs(m00) > DBL_EPSILON) {
        const double inv_m00 = 1. / m00;
        mcx = m10 * inv_m00;
        mcy = m01 * inv_m00;
    }
    const double mu20 = m20 - m10 * mcx;
    const double mu11 = m11 - m10 * mcy;
    const double mu02 = m02 - m01 * mcy;
    if (m00 == 0) {
        *cx = nan; *cy = nan; *orient = nan; *ax0 = nan; *ax1 = nan;
        return;
    }
    const double num = 2 * mu11;
    const double den = mu20 - mu02;
    const double common = sqrt(4 * (mu11 * mu11) + den * den);
    *orient = -.5 * atan2(num, den);
    *cx = m10 / m00;
    *cy = m01 / m00;
    const double k = 2 * sqrt(2.0);
    *ax0 = k * sqrt((mu20 + mu02 + common) / m00);
    *ax1 = k * sqrt((mu20 + mu02 - common) / m00);
}

/* get_frame_features(frames, frame_threshold=thr, mask=mask, use_cc=*) for
 * uint8 frames: use_cc is a no-op for uint8 input (frames > -30 is all-true,
 * M/proc/proc.py:280), so the blob mask is (frame > thr) & mask.
 * area_out (optional) receives contourArea of the selected contour. */
void orc_frame_features(const uint8_t *frames, const uint8_t *mask, int64_t n, int H, int W,
                        double thr, double *centroid, double *orient, double *axes, double *area_out)
{
    const int PW = W + 2, PH = H + 2;
    uint8_t *img = (uint8_t *)calloc((size_t)PW * PH, 1);
    int32_t *lab = (int32_t *)malloc(sizeof(int32_t) * (size_t)PW * PH);
    int32_t *stack = (int32_t *)malloc(sizeof(int32_t) * (size_t)PW * PH);
    for (int64_t f = 0; f < n; ++f) {
        const uint8_t *fr = frames + f * (int64_t)H * W;
        const uint8_t *mk = mask ? mask + f * (int64_t)H * W : NULL;
        memset(img, 0, (size_t)PW * PH);
        for (int y = 0; y < H; ++y)
            for (int x = 0; x < W; ++x)
                img[(y + 1) * PW + (x + 1)] = ((double)fr[y * W + x] > thr) && (!mk || mk[y * W + x]);
        for (int i = 0; i < PW * PH; ++i) lab[i] = 0;
        /* 8-connected components in raster order of their first pixel; the
         * first pixel of a component always starts its outer border. */
        double best_area = -1.0; green_t best = {0, 0, 0, 0, 0, 0}; int found = 0;
        int nlab = 0;
        for (int y = 1; y <= H; ++y)
            for (int x = 1; x <= W; ++x) {
                const int idx = y * PW + x;
                if (!img[idx] || lab[idx]) continue;
                ++nlab;
                int sp = 0; stack[sp++] = idx; lab[idx] = nlab;
                while (sp) {
                    const int c = stack[--sp];
                    const int cy = c / PW, cx = c % PW;
                    for (int d = 0; d < 8; ++d) {
                        const int q = (cy + CDY[d]) * PW + (cx + CDX[d]);
                        if (img[q] && !lab[q]) { lab[q] = nlab; stack[sp++] = q; }
                    }
                }
                const green_t g = trace_outer(img, PW, x, y);
                /* cv::contourArea = |a00| / 2 (oriented=false) */
                const double a = fabs((double)g.a00 * 0.5);
                if (a > best_area) { best_area = a; best = g; found = 1; }
            }
        double cx = NAN, cy = NAN, o = NAN, a0 = NAN, a1 = NAN;
        if (found) moments_to_features(&best, &cx, &cy, &o, &a0, &a1);
        centroid[2 * f] = cx; centroid[2 * f + 1] = cy;
        orient[f] = o; axes[2 * f] = a0; axes[2 * f + 1] = a1;
        if (area_out) area_out[f] = found ? best_area : NAN;
    }
    free(img); free(lab); free(stack);
}

/* ------------------------------------------------------------------ */
/* crop_and_rotate_frame                                               */
/* ------------------------------------------------------------------ */
static inline int cv_round(double v) { return (int)lrint(v); }

/* writes the 80x80 (cw x ch) crop of one uint8 frame */
static void crop_rotate_one(const uint8_t *src, int H, int W, double cxc, double cyc,
                            double angle, int cw, int ch, uint8_t *dst)
{
    memset(dst, 0, (size_t)cw * ch);
    if (isnan(angle) || isnan(cxc) || isnan(cyc)) return;
    if (cxc < 0 || cyc < 0) return;
    /* int() truncates toward zero */
    const int xmin = (int)(cxc - cw / 2) + cw;
    const int xmax = (int)(cxc + cw / 2) + cw;
    const int ymin = (int)(cyc - ch / 2) + ch;
    const int ymax = (int)(cyc + ch / 2) + ch;
    /* copyMakeBorder(frame, top=ch, bottom=ch, left=cw, right=cw) */
    const int PWd = W + 2 * cw, PHd = H + 2 * ch;
    /* numpy slice use_frame[ymin:ymax, xmin:xmax] clamps to the array */
    const int sx0 = xmin < 0 ? 0 : (xmin > PWd ? PWd : xmin);
    const int sx1 = xmax < 0 ? 0 : (xmax > PWd ? PWd : xmax);
    const int sy0 = ymin < 0 ? 0 : (ymin > PHd ? PHd : ymin);
    const int sy1 = ymax < 0 ? 0 : (ymax > PHd ? PHd : ymax);
    const int pw = sx1 - sx0, ph = sy1 - sy0;
    if (pw <= 0 || ph <= 0) return; /* warpAffine raises -> zeros */

    /* getRotationMatrix2D((cw//2, ch//2), angle, 1) */
    const double CV_PI_ = 3.1415926535897932384626433832795;
    const double ang = angle * (CV_PI_ / 180);
    const double alpha = cos(ang) * 1.0, beta = sin(ang) * 1.0;
    const double ccx = (double)(float)(cw / 2), ccy = (double)(float)(ch / 2);
    double M[6] = {alpha, beta, (1 - alpha) * ccx - beta * ccy,
                   -beta, alpha, beta * ccx + (1 - alpha) * ccy};
    /* warpAffine inverts the map (no WARP_INVERSE_MAP) */
    {
        double D = M[0] * M[4] - M[1] * M[3];
        D = D != 0 ? 1. / D : 0;
        const double A11 = M[4] * D, A22 = M[0] * D;
        M[0] = A11; M[1] *= -D;
        M[3] *= -D; M[4] = A22;
        const double b1 = -M[0] * M[2] - M[1] * M[5];
        const double b2 = -M[3] * M[2] - M[4] * M[5];
        M[2] = b1; M[5] = b2;
    }
    const int AB_BITS = 10, AB_SCALE = 1 << AB_BITS, INTER_BITS = 5, INTER_TAB_SIZE = 1 << INTER_BITS;
    const int round_delta = AB_SCALE / INTER_TAB_SIZE / 2;
    for (int y = 0; y < ch; ++y) {
        const int X0 = cv_round((M[1] * y + M[2]) * AB_SCALE) + round_delta;
        const int Y0 = cv_round((M[4] * y + M[5]) * AB_SCALE) + round_delta;
        for (int x = 0; x < cw; ++x) {
            const int adelta = cv_round(M[0] * x * AB_SCALE);
            const int bdelta = cv_round(M[3] * x * AB_SCALE);
            const int X = (X0 + adelta) >> (AB_BITS - INTER_BITS);
            const int Y = (Y0 + bdelta) >> (AB_BITS - INTER_BITS);
            const int sx = X >> INTER_BITS, sy = Y >> INTER_BITS; /* saturate_cast<short>: in range here */
            const int tx = X & (INTER_TAB_SIZE - 1), ty = Y & (INTER_TAB_SIZE - 1);
            /* INTER_LINEAR fixed-point weights (sum == 32768 exactly) */
            const int w0 = (32 - ty) * (32 - tx) * 32, w1 = (32 - ty) * tx * 32;
            const int w2 = ty * (32 - tx) * 32, w3 = ty * tx * 32;
            int v[4];
            for (int t = 0; t < 4; ++t) {
                const int qx = sx + (t & 1), qy = sy + (t >> 1);
                int val = 0; /* BORDER_CONSTANT, value 0 */
                if (qx >= 0 && qx < pw && qy >= 0 && qy < ph) {
                    const int fx = sx0 + qx - cw, fy = sy0 + qy - ch; /* padded -> frame */
                    if (fx >= 0 && fx < W && fy >= 0 && fy < H) val = src[fy * W + fx];
                }
                v[t] = val;
            }
            int acc = v[0] * w0 + v[1] * w1 + v[2] * w2 + v[3] * w3;
            acc = (acc + (1 << 14)) >> 15;
            dst[y * cw + x] = (uint8_t)(acc < 0 ? 0 : (acc > 255 ? 255 : acc));
        }
    }
}

void orc_crop_rotate(const uint8_t *src, int64_t n, int H, int W, const double *center,
                     const double *angle, int cw, int ch, uint8_t *dst)
{
    for (int64_t f = 0; f < n; ++f)
        crop_rotate_one(src + f * (int64_t)H * W, H, W, center[2 * f], center[2 * f + 1],
                        angle[f], cw, ch, dst + f * (int64_t)cw * ch);
}

/* ------------------------------------------------------------------ */
/* cv2.inpaint(img, mask, 3, cv2.INPAINT_NS)                           */
/* ------------------------------------------------------------------ */
#define KNOWN 0
#define BAND 1
#define INSIDE 2

typedef struct { float T; int64_t seq; int i, j; } hent_t;
typedef struct { hent_t *a; int64_t n, cap, seq; } heap_t;

/* OpenCV's CvPriorityQueueFloat is a sorted list: Push inserts after every
 * element with T' <= T, Pop takes the head.  That is a min-heap on (T, seq). */
static inline int hless(const hent_t *x, const hent_t *y)
{ return x->T < y->T || (x->T == y->T && x->seq < y->seq); }
static void hpush(heap_t *h, int i, int j, float T)
{
    hent_t e = {T, h->seq++, i, j};
    int64_t k = h->n++;
    while (k > 0) {
        int64_t p = (k - 1) / 2;
        if (!hless(&e, &h->a[p])) break;
        h->a[k] = h->a[p]; k = p;
    }
    h->a[k] = e;
}
static int hpop(heap_t *h, int *i, int *j)
{
    if (h->n == 0) return 0;
    *i = h->a[0].i; *j = h->a[0].j;
    hent_t e = h->a[--h->n];
    int64_t k = 0;
    for (;;) {
        int64_t c = 2 * k + 1;
        if (c >= h->n) break;
        if (c + 1 < h->n && hless(&h->a[c + 1], &h->a[c])) ++c;
        if (!hless(&h->a[c], &e)) break;
        h->a[k] = h->a[c]; k = c;
    }
    if (h->n > 0) h->a[k] = e;
    return 1;
}

static float fm_solve(int i1, int j1, int i2, int j2, const uint8_t *f, const float *t, int PW)
{
    double sol;
    const double a11 = t[i1 * PW + j1], a22 = t[i2 * PW + j2];
    const double m12 = a11 < a22 ? a11 : a22;
    if (f[i1 * PW + j1] != INSIDE) {
        if (f[i2 * PW + j2] != INSIDE) {
            if (fabs(a11 - a22) >= 1.0) sol = 1 + m12;
            else sol = (a11 + a22 + sqrt((double)(2 - (a11 - a22) * (a11 - a22)))) * 0.5;
        } else sol = 1 + a11;
    } else if (f[i2 * PW + j2] != INSIDE) sol = 1 + a22;
    else sol = 1 + m12;
    return (float)sol;
}

static inline float min4f(float a, float b, float c, float d)
{ float x = a < b ? a : b, y = c < d ? c : d; return x < y ? x : y; }

/* Returns 0 on success.  out may alias img. */
int orc_inpaint_ns_one(const uint8_t *img, const uint8_t *mask, int H, int W, int range, uint8_t *out)
{
    const int PH = H + 2, PW = W + 2;
    uint8_t *f = (uint8_t *)malloc((size_t)PH * PW);
    uint8_t *mp = (uint8_t *)calloc((size_t)PH * PW, 1);
    float *t = (float *)malloc(sizeof(float) * (size_t)PH * PW);
    if (out != img) memcpy(out, img, (size_t)H * W);
    int64_t nmask = 0;
    for (int y = 0; y < H; ++y)
        for (int x = 0; x < W; ++x)
            if (mask[y * W + x]) { mp[(y + 1) * PW + x + 1] = 1; ++nmask; }
    if (nmask == 0) { free(f); free(mp); free(t); return 0; }
    heap_t h; h.cap = (int64_t)PH * PW; h.n = 0; h.seq = 0;
    h.a = (hent_t *)malloc(sizeof(hent_t) * (size_t)h.cap);
    for (int i = 0; i < PH * PW; ++i) { f[i] = KNOWN; t[i] = 1.0e6f; }
    /* band = dilate(mask, 3x3 cross) - mask, zero frame; pushed in raster order */
    for (int i = 1; i < PH - 1; ++i)
        for (int j = 1; j < PW - 1; ++j) {
            const int k = i * PW + j;
            if (mp[k]) { f[k] = INSIDE; continue; }
            if (mp[k - 1] || mp[k + 1] || mp[k - PW] || mp[k + PW]) {
                f[k] = BAND; t[k] = 0.0f;
                hpush(&h, i, j, 0.0f);
            }
        }
    int ii, jj;
    while (hpop(&h, &ii, &jj)) {
        f[ii * PW + jj] = KNOWN;
        for (int q = 0; q < 4; ++q) {
            int i, j;
            if (q == 0) { i = ii - 1; j = jj; }
            else if (q == 1) { i = ii; j = jj - 1; }
            else if (q == 2) { i = ii + 1; j = jj; }
            else { i = ii; j = jj + 1; }
            if (i <= 1 || j <= 1 || i > PH - 1 || j > PW - 1) continue;
            if (f[i * PW + j] != INSIDE) continue;
            const float dist = min4f(fm_solve(i - 1, j, i, j - 1, f, t, PW), fm_solve(i + 1, j, i, j - 1, f, t, PW),
                                     fm_solve(i - 1, j, i, j + 1, f, t, PW), fm_solve(i + 1, j, i, j + 1, f, t, PW));
            t[i * PW + j] = dist;
            float Ia = 0, s = 1.0e-20f;
            for (int k = i - range; k <= i + range; ++k) {
                const int km = k - 1 + (k == 1), kp = k - 1 - (k == PH - 2);
                for (int l = j - range; l <= j + range; ++l) {
                    const int lm = l - 1 + (l == 1), lp = l - 1 - (l == PW - 2);
                    if (!(k > 0 && l > 0 && k < PH - 1 && l < PW - 1)) continue;
                    if (f[k * PW + l] == INSIDE) continue;
                    if ((l - j) * (l - j) + (k - i) * (k - i) > range * range) continue;
                    const float ry = (float)(k - i), rx = (float)(l - j);
                    const float lr = rx * rx + ry * ry;
                    const float dst = (float)(1. / (lr * sqrt((double)lr)));
                    float gx, gy;
                    const int up_ok = f[(k - 1) * PW + l] != INSIDE, dn_ok = f[(k + 1) * PW + l] != INSIDE;
                    const int lf_ok = f[k * PW + l - 1] != INSIDE, rt_ok = f[k * PW + l + 1] != INSIDE;
                    if (dn_ok) {
                        if (up_ok) gx = (float)(abs(out[(kp + 1) * W + lm] - out[kp * W + lm]) +
                                                abs(out[kp * W + lm] - out[(km - 1) * W + lm]));
                        else gx = (float)(abs(out[(kp + 1) * W + lm] - out[kp * W + lm])) * 2.0f;
                    } else {
                        if (up_ok) gx = (float)(abs(out[kp * W + lm] - out[(km - 1) * W + lm])) * 2.0f;
                        else gx = 0;
                    }
                    if (rt_ok) {
                        if (lf_ok) gy = -(float)(abs(out[km * W + lp + 1] - out[km * W + lm]) +
                                                 abs(out[km * W + lm] - out[km * W + lm - 1]));
                        else gy = -(float)(abs(out[km * W + lp + 1] - out[km * W + lm])) * 2.0f;
                    } else {
                        if (lf_ok) gy = -(float)(abs(out[km * W + lm] - out[km * W + lm - 1])) * 2.0f;
                        else gy = 0;
                    }
                    const float dot = rx * gx + ry * gy;
                    const float lg = gx * gx + gy * gy;
                    float dir = fabsf(dot / sqrtf(lr * lg));
                    if (!(dir > 0.01f)) dir = 0.000001f; /* also catches 0/0 (flat) */
                    const float w = dst * dir;
                    Ia += w * (float)out[km * W + lm];
                    s += w;
                }
            }
            const double v = (double)Ia / s;
            int r = (int)lrint(v);
            out[(i - 1) * W + (j - 1)] = (uint8_t)(r < 0 ? 0 : (r > 255 ? 255 : r));
            f[i * PW + j] = BAND;
            hpush(&h, i, j, dist);
        }
    }
    free(h.a); free(f); free(mp); free(t);
    return 0;
}

void orc_inpaint_ns(const uint8_t *img, const uint8_t *mask, int64_t n, int H, int W, int range, uint8_t *out)
{
    for (int64_t f = 0; f < n; ++f)
        orc_inpaint_ns_one(img + f * (int64_t)H * W, mask + f * (int64_t)H * W, H, W, range,
                           out + f * (int64_t)H * W);
}
