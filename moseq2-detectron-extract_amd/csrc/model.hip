// Model handle: the Mask/Keypoint R-CNN forward as one C call.
//
// mdx_model_create parses a Detectron2 state dict (the "MDXW" blob, include/
// mdx.h), folds FrozenBN into the convolutions and packs every weight once
// into the layout its kernel reads (OHWI, fp16 when asked; the stem as a 4x4
// conv over the space-to-depth input; the box head's fc1 columns permuted to
// the NHWC pooled layout; the mask deconv as a 4*Co-column GEMM with a
// pixel-shuffle epilogue; the keypoint deconv as a GEMM + col2im).
//
// mdx_model_forward enqueues the whole eval-mode GeneralizedRCNN inference of
// the reference (M/model/predict.py:92 -> Detectron2, configured by
// M/model/config.py:21-94) on one stream: preprocess (scale LUT, 1->3
// replication, normalisation, pad to /32) -> ResNet -> FPN (GN, avg fuse,
// P6) -> RPN (top-k, decode, NMS, merge) -> ROIAlignV2 -> box head + fast R-CNN
// inference -> mask head + paste -> keypoint head + heatmaps_to_keypoints.
// Fixed shapes (post-NMS-topk proposals and D detections per image, counts on
// the device) mean no host synchronisation, so a reserved forward can be
// captured into a HIP graph.  Every intermediate lives in a per-stream arena:
// one allocation sized by a dry run of the same code, bump-allocated per
// forward, so forwards on different streams run concurrently.
#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <unordered_map>
#include <vector>

#include "common.h"

namespace mdx {
namespace {

constexpr int64_t SPLITK_WS = 64ll << 20;  // fp32 partials of split-K launches

struct HostT {
    std::vector<int64_t> shape;
    std::vector<float> v;
    int64_t numel() const {
        int64_t n = 1;
        for (auto d : shape) n *= d;
        return n;
    }
};

struct ConvW {
    void *w = nullptr;
    float *b = nullptr;
    int cin = 0, cout = 0, k = 1, stride = 1, pad = 0, kalg = 0;
    int dt = 0;  // operand / activation dtype of the layer: 0 f32, 1 f16
    // Winograd weights U = G g G^T of F(2x2,3x3) [16][Cout][Cin] and F(4x4,3x3)
    // [36][Cout][Cin] (fp32 3x3/s1/p1 layers with Cin >= 128)
    float *wino2 = nullptr, *wino4 = nullptr, *wino6 = nullptr;
    // the same U split into bf16 planes (split-plane mode handles):
    // winox6[m / 2 - 1] for F(m x m, 3x3)
    void *winox6[3] = {nullptr, nullptr, nullptr};
    // fp32 Linear layers: the weights split once into bf16 planes for
    // mdx_gemm_x6 (used while mdx_policy.fp32_split != 0)
    void *x6 = nullptr;
    // fp32 conv layers of split-plane handles (KH*KW*Cin % 32 == 0): the OHWI
    // weights as bf16 planes, k_conv_x3's pre-split B operand
    void *wp = nullptr;
};

struct GnW {
    float *g = nullptr, *b = nullptr;
};

struct Block {
    int stage;
    bool has_sc;
    ConvW sc, c1, c2, c3;
    // conv3 and the projection shortcut as one GEMM over K = Cin3 + Cin_sc
    // (mdx_conv2d_dual; packed when mdx_policy.fuse_shortcut is on)
    ConvW c3sc;
};

struct TensorRec {
    void *p;
    int64_t shape[4];
    int dtype;
    int64_t offset;  // bytes from the arena base (-1: caller-owned)
};

struct ProfEv {
    hipEvent_t e0, e1;
    mdx_conv_record r;
};

struct Ctx {
    char *base = nullptr;
    size_t cap = 0, off = 0;
    bool dry = false;
    std::map<std::string, TensorRec> named;
    std::vector<ProfEv> prof;
    // Winograd scratch (V and M of one layer at a time, stream-ordered):
    // sized by the dry run's largest layer, allocated by reserve()
    char *wino_base = nullptr;
    size_t wino_cap = 0, wino_need = 0;
    void *alloc(size_t bytes) {
        off = (off + 255) & ~(size_t)255;
        void *p = base + off;
        off += bytes;
        return dry ? (void *)(uintptr_t)(0x1000 + off) : p;  // dry: a non-null placeholder, never dereferenced
    }
};

struct Model {
    mdx_model_cfg cfg{};
    int dev = 0;
    int dt = 0;        // 0 f32, 1 f16 (backbone, FPN, RPN, box head)
    int hdt = 0;       // mask + keypoint heads (cfg.head_dtype; = dt unless mixed)
    bool stem_fold = false;  // stem over the 2-channel (value, inside) s2d input (fp32 handles)
    bool fuse_sc = false;    // projection shortcuts fused into conv3 (Block::c3sc)
    // the Winograd policy and fp32 split mode the weights were prepared for
    // (Winograd U tiles, bf16 planes): a later switch runs the layers it did
    // not prepare on the fallback kernels, reported once
    // the kernel-selection policy of this handle (captured from the creating
    // thread at mdx_model_create; installed on the calling thread by every
    // entry point that packs or runs the forward, PolicyScope)
    mdx_policy policy{};
    size_t es = 4;     // activation element size
    std::vector<void *> allocs;
    ConvW stem;
    std::vector<Block> blocks;
    ConvW fpn_lat[4], fpn_out[4];
    GnW gn_lat[4], gn_out[4];
    ConvW rpn_conv, rpn_head;
    std::vector<float> cell_anchors;  // [L][A][4]
    std::vector<ConvW> fc;
    ConvW box_pred;
    std::vector<ConvW> mask_convs;
    ConvW mask_deconv, mask_pred;
    std::vector<ConvW> kp_convs;
    ConvW kp_deconv;
    float *kp_deconv_b = nullptr;
    std::mutex mu;
    std::map<hipStream_t, std::unique_ptr<Ctx>> ctx;
    bool profile = false;
    std::vector<mdx_conv_record> last_prof;
    ~Model() {
        for (auto &kv : ctx) {
            if (kv.second->base) (void)hipFree(kv.second->base);
            if (kv.second->wino_base) (void)hipFree(kv.second->wino_base);
            for (auto &p : kv.second->prof) {
                (void)hipEventDestroy(p.e0);
                (void)hipEventDestroy(p.e1);
            }
        }
        for (void *p : allocs) (void)hipFree(p);
    }
};

// ------------------------------------------------------------ blob parsing
bool parse_blob(const void *blob, int64_t nbytes, std::unordered_map<std::string, HostT> &sd) {
    const char *p = (const char *)blob, *end = p + nbytes;
    auto take = [&](void *dst, size_t n) -> bool {
        if (p + n > end) return false;
        memcpy(dst, p, n);
        p += n;
        return true;
    };
    char magic[4];
    uint32_t version, count;
    if (!take(magic, 4) || memcmp(magic, "MDXW", 4) != 0) {
        set_error("mdx_model_create: weights blob does not start with \"MDXW\"");
        return false;
    }
    if (!take(&version, 4) || version != 1 || !take(&count, 4)) {
        set_error("mdx_model_create: unsupported weights blob version");
        return false;
    }
    for (uint32_t i = 0; i < count; ++i) {
        uint32_t nl, nd;
        if (!take(&nl, 4) || nl > 4096 || p + nl > end) {
            set_error("mdx_model_create: truncated weights blob (entry %u)", i);
            return false;
        }
        std::string name(p, nl);
        p += nl;
        HostT t;
        if (!take(&nd, 4) || nd > 8) {
            set_error("mdx_model_create: bad rank for %s", name.c_str());
            return false;
        }
        t.shape.resize(nd);
        if (nd && !take(t.shape.data(), 8 * nd)) {
            set_error("mdx_model_create: truncated shape of %s", name.c_str());
            return false;
        }
        const int64_t n = t.numel();
        if (n < 0 || p + 4 * n > end) {
            set_error("mdx_model_create: truncated data of %s", name.c_str());
            return false;
        }
        t.v.resize((size_t)n);
        memcpy(t.v.data(), p, 4 * (size_t)n);
        p += 4 * n;
        sd[name] = std::move(t);
    }
    return true;
}

// fp32 -> fp16 round to nearest even (the device conversion)
inline uint16_t f2h(float f) {
    _Float16 h = (_Float16)f;
    uint16_t u;
    memcpy(&u, &h, 2);
    return u;
}

struct Packer {
    Model &m;
    std::unordered_map<std::string, HostT> &sd;
    std::string err;
    int cur_dt = 0;  // dtype of the layers being packed (m.dt, or m.hdt for the mask / keypoint heads)

    const HostT *get(const std::string &k, std::initializer_list<int64_t> shape = {}) {
        auto it = sd.find(k);
        if (it == sd.end()) {
            if (err.empty()) err = "missing weight \"" + k + "\"";
            return nullptr;
        }
        if (shape.size()) {
            std::vector<int64_t> s(shape);
            bool ok = s.size() == it->second.shape.size();
            for (size_t i = 0; ok && i < s.size(); ++i) ok = s[i] < 0 || s[i] == it->second.shape[i];
            if (!ok) {
                if (err.empty()) err = "weight \"" + k + "\" has an unexpected shape";
                return nullptr;
            }
        }
        return &it->second;
    }
    bool has(const std::string &k) const { return sd.count(k) != 0; }

    void *upload(const std::vector<float> &v, bool as_act_dtype) {
        if (!err.empty()) return nullptr;
        void *d = nullptr;
        const bool h = as_act_dtype && cur_dt == 1;
        const size_t bytes = v.size() * (h ? 2 : 4);
        if (hipMalloc(&d, bytes ? bytes : 4) != hipSuccess) {
            err = "device allocation of weights failed";
            return nullptr;
        }
        m.allocs.push_back(d);
        if (h) {
            std::vector<uint16_t> hv(v.size());
            for (size_t i = 0; i < v.size(); ++i) hv[i] = f2h(v[i]);
            if (hipMemcpy(d, hv.data(), bytes, hipMemcpyHostToDevice) != hipSuccess) err = "weight upload failed";
        } else if (bytes) {
            if (hipMemcpy(d, v.data(), bytes, hipMemcpyHostToDevice) != hipSuccess) err = "weight upload failed";
        }
        return d;
    }
    float *upload_f32(const std::vector<float> &v) { return (float *)upload(v, false); }
    // device fp32 rows x K (K % 16 == 0) -> bf16 planes (mdx_split_x6 layout), owned by the model
    void *split_planes(const float *w, int64_t rows, int K) {
        void *d = nullptr;
        if (hipMalloc(&d, (size_t)mdx_x6_plane_bytes(rows, K)) != hipSuccess) {
            err = "device allocation of weight planes failed";
            return nullptr;
        }
        m.allocs.push_back(d);
        if (mdx_split_x6(w, rows, K, K, d, nullptr) != MDX_OK || hipDeviceSynchronize() != hipSuccess) {
            err = "weight plane split failed";
            return nullptr;
        }
        return d;
    }

    // Winograd tile sizes to pack for the next 3x3 layers: the ones the
    // policy current at create time can pick (mdx_winograd_tile); the heads
    // set the map size they run on (map_hw > 0), the trunk leaves it 0 (any
    // size: F(6,3) and F(4,3) under policy 6).  A mode switched later to a
    // size that was not packed runs those layers direct.
    int map_hw = 0;
    bool want_tile(int m_) const {
        const int wp = pol().winograd;
        if (wp == 0) return false;
        if (map_hw > 0) return mdx_winograd_tile(map_hw, map_hw, wp) == m_;
        return wp == 6 ? (m_ == 4 || m_ == 6) : wp == m_;
    }
    // OIHW (optionally scaled per output channel) -> [Cout][KH][KW][Cin]
    ConvW conv(const HostT *w, const float *scale, const std::vector<float> *bias, int stride, int pad) {
        ConvW c;
        if (!w || w->shape.size() != 4) {
            if (err.empty()) err = "conv weight must be 4-D";
            return c;
        }
        const int co = (int)w->shape[0], ci = (int)w->shape[1], kh = (int)w->shape[2], kw = (int)w->shape[3];
        std::vector<float> p((size_t)co * kh * kw * ci);
        for (int o = 0; o < co; ++o)
            for (int i = 0; i < ci; ++i)
                for (int y = 0; y < kh; ++y)
                    for (int x = 0; x < kw; ++x) {
                        float v = w->v[(((size_t)o * ci + i) * kh + y) * kw + x];
                        if (scale) v *= scale[o];
                        p[(((size_t)o * kh + y) * kw + x) * ci + i] = v;
                    }
        c.w = upload(p, true);
        if (bias) c.b = upload_f32(*bias);
        c.cin = ci;
        c.cout = co;
        c.k = kh;
        c.stride = stride;
        c.pad = pad;
        c.dt = cur_dt;
        if (cur_dt == 0 && pol().fp32_split == 6 && ((size_t)kh * kw * ci) % 32 == 0 && c.w && err.empty()) {
            c.wp = split_planes((const float *)c.w, co, kh * kw * ci);
            if (!c.wp) return c;
        }
        if (cur_dt == 0 && kh == 3 && kw == 3 && stride == 1 && pad == 1 && ci >= 64 && ci % 4 == 0 && co % 8 == 0 &&
            err.empty()) {
            std::vector<float> oihw((size_t)co * ci * 9), u;
            for (int o = 0; o < co; ++o)
                for (size_t q = 0; q < (size_t)ci * 9; ++q)
                    oihw[(size_t)o * ci * 9 + q] = w->v[(size_t)o * ci * 9 + q] * (scale ? scale[o] : 1.f);
            for (int m_ : {2, 4, 6}) {
                if (!want_tile(m_)) continue;
                const int nb = (m_ + 2) * (m_ + 2);
                u.resize((size_t)nb * co * ci);
                mdx_winograd_weights(oihw.data(), co, ci, m_, u.data());
                float *ud = upload_f32(u);
                (m_ == 2 ? c.wino2 : m_ == 4 ? c.wino4 : c.wino6) = ud;
                // split-plane handles: U as bf16 planes too (the pre-split B
                // operand of k_conv_x3, or k_gemm_x6's with MDX_WINO_X6)
                if (pol().fp32_split == 6 && ci % 16 == 0 && ud && err.empty()) {
                    c.winox6[m_ / 2 - 1] = split_planes(ud, (int64_t)nb * co, ci);
                    if (!c.winox6[m_ / 2 - 1]) break;
                }
            }
        }
        return c;
    }
    // FrozenBatchNorm2d folded: scale = w * rsqrt(var + eps), bias = b - mean * scale
    void bn(const std::string &p, int c, std::vector<float> &scale, std::vector<float> &bias) {
        const HostT *g = get(p + ".norm.weight", {c}), *b = get(p + ".norm.bias", {c});
        const HostT *mu = get(p + ".norm.running_mean", {c}), *var = get(p + ".norm.running_var", {c});
        scale.assign(c, 1.f);
        bias.assign(c, 0.f);
        if (!g || !b || !mu || !var) return;
        for (int i = 0; i < c; ++i) {
            scale[i] = g->v[i] * (1.0f / std::sqrt(var->v[i] + 1e-5f));
            bias[i] = b->v[i] - mu->v[i] * scale[i];
        }
    }
    ConvW conv_bn(const std::string &p, int stride, int pad) {
        const HostT *w = get(p + ".weight");
        if (!w) return {};
        std::vector<float> s, b;
        bn(p, (int)w->shape[0], s, b);
        return conv(w, s.data(), &b, stride, pad);
    }
    // conv3 (1x1, Cin3 -> Cout) and shortcut (1x1 / stride s, Cin_sc -> Cout),
    // both FrozenBN-folded, as one [Cout][Cin3 + Cin_sc] matrix, bias b3 + b_sc
    ConvW conv3_shortcut(const std::string &p3, const std::string &psc, int stride) {
        const HostT *w3 = get(p3 + ".weight"), *ws = get(psc + ".weight");
        ConvW c;
        if (!w3 || !ws) return c;
        if (w3->shape.size() != 4 || ws->shape.size() != 4 || w3->shape[2] != 1 || w3->shape[3] != 1 ||
            ws->shape[2] != 1 || ws->shape[3] != 1 || w3->shape[0] != ws->shape[0]) {
            if (err.empty()) err = "conv3 / shortcut must be 1x1 convs with the same Cout";
            return c;
        }
        const int co = (int)w3->shape[0], c3 = (int)w3->shape[1], cs = (int)ws->shape[1];
        std::vector<float> s3, b3, ss, bs;
        bn(p3, co, s3, b3);
        bn(psc, co, ss, bs);
        std::vector<float> pk((size_t)co * (c3 + cs)), b(co);
        for (int o = 0; o < co; ++o) {
            for (int i = 0; i < c3; ++i) pk[(size_t)o * (c3 + cs) + i] = w3->v[(size_t)o * c3 + i] * s3[o];
            for (int i = 0; i < cs; ++i) pk[(size_t)o * (c3 + cs) + c3 + i] = ws->v[(size_t)o * cs + i] * ss[o];
            b[o] = b3[o] + bs[o];
        }
        c.w = upload(pk, true);
        c.b = upload_f32(b);
        c.dt = cur_dt;
        c.cin = c3;  // the first source's channels; cout, stride of the second
        c.cout = co;
        c.k = 1;
        c.stride = stride;
        c.kalg = cs;  // (here: the shortcut's Cin)
        return c;
    }
    ConvW conv_plain(const std::string &p, int stride, int pad, bool need_bias) {
        const HostT *w = get(p + ".weight");
        const HostT *b = need_bias ? get(p + ".bias") : (has(p + ".bias") ? get(p + ".bias") : nullptr);
        return conv(w, nullptr, b ? &b->v : nullptr, stride, pad);
    }
    // 7x7/s2/p3 stem -> 4x4/s1/p1 conv over the space-to-depth input
    // (mdx_preprocess_s2d): W'[o][ty][tx][(2dy+dx)*4+c] = W[o][c][2ty+dy][2tx+dx]
    ConvW stem(const std::string &p) {
        const HostT *w = get(p + ".weight");
        ConvW c;
        if (!w) return c;
        if (w->shape.size() != 4 || w->shape[2] != 7 || w->shape[3] != 7 || w->shape[1] > 4) {
            err = "stem must be a 7x7 conv over <= 4 channels";
            return c;
        }
        const int co = (int)w->shape[0], ci = (int)w->shape[1];
        std::vector<float> s, b;
        bn(p, co, s, b);
        if (m.stem_fold) {
            // every input channel is the same scaled pixel v, normalised per
            // channel and zero outside the image: sum_c w_c (v - mean_c) /
            // std_c = (sum_c w_c / std_c) v - (sum_c w_c mean_c / std_c) [inside]
            // -> 2 channels (v, inside) per s2d phase, K = 4 x 4 x 8 (double sums, one rounding)
            std::vector<float> pk((size_t)co * 128, 0.f);
            for (int o = 0; o < co; ++o)
                for (int ky = 0; ky < 7; ++ky)
                    for (int kx = 0; kx < 7; ++kx) {
                        double wv = 0, wi = 0;
                        for (int ch = 0; ch < ci; ++ch) {
                            const double wt = (double)w->v[(((size_t)o * ci + ch) * 7 + ky) * 7 + kx] * s[o];
                            wv += wt / m.cfg.pixel_std[ch];
                            wi -= wt * m.cfg.pixel_mean[ch] / m.cfg.pixel_std[ch];
                        }
                        const int ty = ky >> 1, dy = ky & 1, tx = kx >> 1, dx = kx & 1;
                        const size_t q = (size_t)o * 128 + ((ty * 4 + tx) * 4 + dy * 2 + dx) * 2;
                        pk[q] = (float)wv;
                        pk[q + 1] = (float)wi;
                    }
            c.w = upload(pk, true);
            c.b = upload_f32(b);
            c.dt = cur_dt;
            c.cin = 8;
            c.cout = co;
            c.k = 4;
            c.stride = 1;
            c.pad = 1;
            c.kalg = 49 * ci;
            return c;
        }
        std::vector<float> pk((size_t)co * 256, 0.f);
        for (int o = 0; o < co; ++o)
            for (int ch = 0; ch < ci; ++ch)
                for (int ky = 0; ky < 7; ++ky)
                    for (int kx = 0; kx < 7; ++kx) {
                        const int ty = ky >> 1, dy = ky & 1, tx = kx >> 1, dx = kx & 1;
                        pk[(size_t)o * 256 + ((ty * 4 + tx) * 4 + dy * 2 + dx) * 4 + ch] =
                            w->v[(((size_t)o * ci + ch) * 7 + ky) * 7 + kx] * s[o];
                    }
        c.w = upload(pk, true);
        c.b = upload_f32(b);
        c.dt = cur_dt;
        c.cin = 16;
        c.cout = co;
        c.k = 4;
        c.stride = 1;
        c.pad = 1;
        c.kalg = 49 * ci;
        return c;
    }
    // (out, in) linear as a 1x1 conv
    ConvW linear(const std::vector<float> &w, int out, int in, const std::vector<float> &b, bool x6 = false) {
        ConvW c;
        c.w = upload(w, true);
        c.b = upload_f32(b);
        c.cin = in;
        c.cout = out;
        c.dt = cur_dt;
        if (x6 && cur_dt == 0 && in % 16 == 0 && err.empty()) {
            void *d = nullptr;
            if (hipMalloc(&d, (size_t)mdx_x6_plane_bytes(out, in)) != hipSuccess) {
                err = "device allocation of weight planes failed";
                return c;
            }
            m.allocs.push_back(d);
            if (mdx_split_x6((const float *)c.w, out, in, in, d, nullptr) != MDX_OK ||
                hipDeviceSynchronize() != hipSuccess)
                err = "weight plane split failed";
            c.x6 = d;
        }
        return c;
    }
};

bool pack(Model &m, std::unordered_map<std::string, HostT> &sd, std::string &err) {
    const mdx_model_cfg &cfg = m.cfg;
    Packer P{m, sd, "", m.dt};
    const std::string bu = "backbone.bottom_up";
    m.stem = P.stem(bu + ".stem.conv1");
    const int nb50[4] = {3, 4, 6, 3}, nb101[4] = {3, 4, 23, 3};
    const int *nb = cfg.depth == 50 ? nb50 : nb101;
    for (int st = 0; st < 4; ++st) {
        for (int b = 0; b < nb[st]; ++b) {
            const std::string p = bu + ".res" + std::to_string(st + 2) + "." + std::to_string(b);
            const int s = (b == 0 && st > 0) ? 2 : 1;
            const int s1 = cfg.stride_in_1x1 ? s : 1, s3 = cfg.stride_in_1x1 ? 1 : s;
            Block blk;
            blk.stage = st;
            blk.has_sc = P.has(p + ".shortcut.weight");
            if (blk.has_sc) blk.sc = P.conv_bn(p + ".shortcut", s, 0);
            blk.c1 = P.conv_bn(p + ".conv1", s1, 0);
            blk.c2 = P.conv_bn(p + ".conv2", s3, 1);
            blk.c3 = P.conv_bn(p + ".conv3", 1, 0);
            if (blk.has_sc && m.fuse_sc) blk.c3sc = P.conv3_shortcut(p + ".conv3", p + ".shortcut", s);
            m.blocks.push_back(blk);
        }
    }
    const int C = cfg.fpn_out_channels;
    for (int l = 0; l < 4; ++l) {
        const std::string lat = "backbone.fpn_lateral" + std::to_string(l + 2);
        const std::string out = "backbone.fpn_output" + std::to_string(l + 2);
        m.fpn_lat[l] = P.conv_plain(lat, 1, 0, false);
        m.fpn_out[l] = P.conv_plain(out, 1, 1, false);
        const HostT *g1 = P.get(lat + ".norm.weight", {C}), *b1 = P.get(lat + ".norm.bias", {C});
        const HostT *g2 = P.get(out + ".norm.weight", {C}), *b2 = P.get(out + ".norm.bias", {C});
        if (g1 && b1 && g2 && b2) {
            m.gn_lat[l] = {P.upload_f32(g1->v), P.upload_f32(b1->v)};
            m.gn_out[l] = {P.upload_f32(g2->v), P.upload_f32(b2->v)};
        }
    }
    const std::string rp = "proposal_generator.rpn_head";
    m.rpn_conv = P.conv_plain(rp + ".conv", 1, 1, true);
    const int A = cfg.n_aspect_ratios;
    {
        const HostT *ow = P.get(rp + ".objectness_logits.weight", {A, C, 1, 1});
        const HostT *ob = P.get(rp + ".objectness_logits.bias", {A});
        const HostT *dw = P.get(rp + ".anchor_deltas.weight", {4 * A, C, 1, 1});
        const HostT *db = P.get(rp + ".anchor_deltas.bias", {4 * A});
        if (ow && ob && dw && db) {
            std::vector<float> w(ow->v), b(ob->v);
            w.insert(w.end(), dw->v.begin(), dw->v.end());
            b.insert(b.end(), db->v.begin(), db->v.end());
            m.rpn_head = P.linear(w, 5 * A, C, b);
        }
    }
    // cell anchors (DefaultAnchorGenerator: computed in double, stored float)
    m.cell_anchors.clear();
    for (int l = 0; l < cfg.n_anchor_sizes; ++l)
        for (int a = 0; a < A; ++a) {
            const double area = (double)cfg.anchor_sizes[l] * (double)cfg.anchor_sizes[l];
            const double w = std::sqrt(area / (double)cfg.aspect_ratios[a]);
            const double h = (double)cfg.aspect_ratios[a] * w;
            m.cell_anchors.insert(m.cell_anchors.end(), {(float)(-w / 2.0), (float)(-h / 2.0), (float)(w / 2.0),
                                                         (float)(h / 2.0)});
        }
    // box head: fc1 columns (c, ry, rx) -> NHWC pooled order (ry, rx, c)
    const int R = cfg.box_pooler_resolution, F = cfg.box_fc_dim;
    {
        int fin = C * R * R;
        for (int i = 0; i < cfg.box_num_fc; ++i) {
            const std::string p = "roi_heads.box_head.fc" + std::to_string(i + 1);
            const HostT *w = P.get(p + ".weight", {F, fin}), *b = P.get(p + ".bias", {F});
            if (!w || !b) break;
            std::vector<float> pw(w->v);
            if (i == 0)
                for (int o = 0; o < F; ++o)
                    for (int c = 0; c < C; ++c)
                        for (int q = 0; q < R * R; ++q)
                            pw[(size_t)o * fin + (size_t)q * C + c] = w->v[(size_t)o * fin + (size_t)c * R * R + q];
            m.fc.push_back(P.linear(pw, F, fin, b->v, true));
            fin = F;
        }
        const int nc = cfg.num_classes;
        const HostT *cw = P.get("roi_heads.box_predictor.cls_score.weight", {nc + 1, F});
        const HostT *cb = P.get("roi_heads.box_predictor.cls_score.bias", {nc + 1});
        const HostT *bw = P.get("roi_heads.box_predictor.bbox_pred.weight", {4 * nc, F});
        const HostT *bb = P.get("roi_heads.box_predictor.bbox_pred.bias", {4 * nc});
        if (cw && cb && bw && bb) {
            std::vector<float> w(cw->v), b(cb->v);
            w.insert(w.end(), bw->v.begin(), bw->v.end());
            b.insert(b.end(), bb->v.begin(), bb->v.end());
            m.box_pred = P.linear(w, 5 * nc + 1, F, b);
        }
    }
    P.cur_dt = m.hdt;  // the mask and keypoint heads (fp16 in the mixed configuration)
    if (cfg.mask_on) {
        P.map_hw = cfg.mask_pooler_resolution;
        for (int i = 0; i < cfg.mask_num_conv; ++i)
            m.mask_convs.push_back(P.conv_plain("roi_heads.mask_head.mask_fcn" + std::to_string(i + 1), 1, 1, true));
        const int cin = cfg.mask_num_conv ? cfg.mask_conv_dim : C, co = cfg.mask_conv_dim;
        const HostT *dw = P.get("roi_heads.mask_head.deconv.weight", {cin, co, 2, 2});
        const HostT *db = P.get("roi_heads.mask_head.deconv.bias", {co});
        if (dw && db) {
            // (Cin, Co, 2, 2) -> row (dy*2+dx)*Co + co, column ci; bias repeated per (dy, dx)
            std::vector<float> w((size_t)4 * co * cin), b((size_t)4 * co);
            for (int ci = 0; ci < cin; ++ci)
                for (int o = 0; o < co; ++o)
                    for (int q = 0; q < 4; ++q) w[((size_t)q * co + o) * cin + ci] = dw->v[((size_t)ci * co + o) * 4 + q];
            for (int q = 0; q < 4; ++q)
                for (int o = 0; o < co; ++o) b[(size_t)q * co + o] = db->v[o];
            m.mask_deconv = P.linear(w, 4 * co, cin, b);
        }
        m.mask_pred = P.conv_plain("roi_heads.mask_head.predictor", 1, 0, true);
    }
    if (cfg.keypoint_on) {
        P.map_hw = cfg.keypoint_pooler_resolution;
        for (int i = 0; i < cfg.n_keypoint_convs; ++i)
            m.kp_convs.push_back(
                P.conv_plain("roi_heads.keypoint_head.conv_fcn" + std::to_string(i + 1), 1, 1, true));
        const int cin = cfg.n_keypoint_convs ? cfg.keypoint_conv_dims[cfg.n_keypoint_convs - 1] : C;
        const int K = cfg.num_keypoints;
        const HostT *kw = P.get("roi_heads.keypoint_head.score_lowres.weight", {cin, K, 4, 4});
        const HostT *kb = P.get("roi_heads.keypoint_head.score_lowres.bias", {K});
        if (kw && kb) {
            // ConvTranspose2d(k4, s2, p1) = GEMM to K*16 columns (k, ky, kx) + col2im
            std::vector<float> w((size_t)K * 16 * cin);
            for (int ci = 0; ci < cin; ++ci)
                for (int k = 0; k < K; ++k)
                    for (int q = 0; q < 16; ++q) w[((size_t)k * 16 + q) * cin + ci] = kw->v[((size_t)ci * K + k) * 16 + q];
            m.kp_deconv = P.linear(w, K * 16, cin, std::vector<float>());
            m.kp_deconv.b = nullptr;
            m.kp_deconv_b = P.upload_f32(kb->v);
        }
    }
    err = P.err;
    return err.empty();
}

// ------------------------------------------------------------ forward
// Winograd layers in image slices (mdx_policy.wino_slice_mb: MB of transformed input per slice;
// 0 = the whole batch in one pass): the input transform, batched GEMM and
// output transform of a slice then move V and M through the 256 MB Infinity
// Cache instead of HBM.  Profiled forwards keep one pass (the probe times
// the three launches of one call).
static int wino_slice_images(int N, int H, int W, int cin, int cout, int m, bool profile) {
    if (pol().wino_slice_mb <= 0 || profile) return N;
    const double tiles = (double)((H + m - 1) / m) * ((W + m - 1) / m);
    const double v = tiles * (m + 2) * (m + 2) * 4.0 * (cin > cout ? cin : cout);  // V or M bytes per image
    const int per = (int)((double)pol().wino_slice_mb * (1 << 20) / v);
    return per < 1 ? 1 : (per >= N ? N : per);
}

struct Fwd {
    Model &m;
    Ctx &c;
    hipStream_t s;
    int rc = MDX_OK;
    void *splitk = nullptr;

    bool ok() const { return rc == MDX_OK; }
    void chk(int r) {
        if (rc == MDX_OK && r != MDX_OK) rc = r;
    }
    void *alloc(size_t bytes) { return c.alloc(bytes); }
    void name(const char *n, void *p, int64_t a, int64_t b, int64_t cc, int64_t d, int dtype) {
        if (c.dry) return;
        const int64_t off = (char *)p >= c.base && (char *)p < c.base + c.cap ? (char *)p - c.base : -1;
        c.named[n] = TensorRec{p, {a, b, cc, d}, dtype, off};
    }
    // conv + bias (+ residual) (+ ReLU); out_mode 1 = 2x2 deconv pixel shuffle
    // in_planes: x is already in the bf16 plane layout (the box pooler's plane output)
    void *conv(const void *x, int N, int H, int W, const ConvW &cw, bool relu, int &OH, int &OW,
               const void *residual = nullptr, bool out_f32 = false, int out_mode = 0, void *out = nullptr,
               bool in_planes = false) {
        OH = (H + 2 * cw.pad - cw.k) / cw.stride + 1;
        OW = (W + 2 * cw.pad - cw.k) / cw.stride + 1;
        const size_t oes = out_f32 ? 4 : (cw.dt == 1 ? 2 : 4);
        // a Linear layer whose A operand passes the 2 GiB range of a buffer
        // descriptor (fp32 box fc1 at B = 64: 64000 x 12544 x 4 B) runs as
        // row slices of the same GEMM
        const size_t ies = cw.dt == 1 ? 2 : 4;
        if (cw.k == 1 && H == 1 && W == 1 && !in_planes && (size_t)N * cw.cin * ies >= (1ull << 31)) {
            if (!out) out = alloc((size_t)N * cw.cout * oes);
            const int rows = (int)(((1ull << 30) / ((size_t)cw.cin * ies)) / 256 * 256);
            for (int r0 = 0; r0 < N; r0 += rows) {
                const int n = std::min(rows, N - r0);
                int oh_, ow_;
                conv((const char *)x + (size_t)r0 * cw.cin * ies, n, 1, 1, cw, relu, oh_, ow_,
                     residual ? (const char *)residual + (size_t)r0 * cw.cout * oes : nullptr, out_f32, out_mode,
                     (char *)out + (size_t)r0 * cw.cout * oes);
            }
            return out;
        }
        if (!out) out = alloc((size_t)N * OH * OW * cw.cout * oes);
        const int wm = mdx_winograd_tile(H, W, pol().winograd);
        const float *wu = wm == 2 ? cw.wino2 : wm == 4 ? cw.wino4 : wm == 6 ? cw.wino6 : nullptr;
        const bool wino = wu && !residual && out_mode == 0 && cw.cin >= pol().winograd_min_cin;
        if (wino) {
            const size_t need = (size_t)mdx_winograd_workspace_bytes(N, H, W, cw.cin, cw.cout, wm);
            if (c.dry) c.wino_need = need > c.wino_need ? need : c.wino_need;
        }
        // fp32 Linear layers in split-plane mode: activations split into bf16
        // planes, GEMM on the bf16 matrix cores (mdx_gemm_x6)
        const bool x6 = cw.x6 && cw.dt == 0 && !out_f32 && out_mode == 0 && cw.k == 1 && cw.stride == 1 &&
                        pol().fp32_split == 6;
        if (in_planes && !x6 && rc == MDX_OK) {
            set_error("model forward: plane input for a layer not in split-plane mode");
            rc = MDX_EINVAL;
        }
        void *planes = x6 && !in_planes ? alloc((size_t)mdx_x6_plane_bytes((int64_t)N * H * W, cw.cin)) : nullptr;
        if (c.dry || !ok()) return out;
        ProfEv *pe = nullptr;
        WinoProbe probe{};
        if (m.profile && wino) {
            for (auto &e : probe.ev) (void)hipEventCreate(&e);
            wino_probe(&probe);
        } else if (m.profile) {
            c.prof.emplace_back();
            pe = &c.prof.back();
            (void)hipEventCreate(&pe->e0);
            (void)hipEventCreate(&pe->e1);
            (void)hipEventRecord(pe->e0, s);
        }
        if (x6) {
            const int64_t rows = (int64_t)N * H * W;
            if (!in_planes) chk(mdx_split_x6((const float *)x, rows, cw.cin, cw.cin, planes, s));
            chk(mdx_gemm_x6(in_planes ? x : planes, cw.x6, cw.b, (int)rows, cw.cout, cw.cin, (const float *)residual, relu ? 1 : 0,
                            (float *)out, s));
        } else if (wino) {
            const void *wx6 = pol().fp32_split == 6 ? cw.winox6[wm / 2 - 1] : nullptr;
            if (wx6 && mdx::winograd_planes_enabled())
                chk(mdx_conv3x3_winograd_x6((const float *)x, N, H, W, cw.cin, wu, wx6, cw.b, cw.cout, relu ? 1 : 0,
                                            wm, (float *)out, c.wino_base, (int64_t)c.wino_cap, s));
            else {
                mdx::x3_weight_planes(wx6);  // the split-plane GEMMs take U's planes (K = Cin % 32 == 0)
                // image slices whose transformed tensors stay in the Infinity
                // Cache between the three launches (mdx_policy.wino_slice_mb)
                const int ns = wino_slice_images(N, H, W, cw.cin, cw.cout, wm, m.profile);
                for (int i0 = 0; i0 < N; i0 += ns) {
                    const int n = std::min(ns, N - i0);
                    chk(mdx_conv3x3_winograd((const float *)x + (size_t)i0 * H * W * cw.cin, n, H, W, cw.cin, wu, cw.b,
                                             cw.cout, relu ? 1 : 0, wm, (float *)out + (size_t)i0 * OH * OW * cw.cout,
                                             c.wino_base, (int64_t)c.wino_cap, s));
                }
                mdx::x3_weight_planes(nullptr);
            }
            if (m.profile) {
                wino_probe(nullptr);
                // three records: input transform, batched GEMM, output transform
                const int64_t A = wm + 2, T = (int64_t)N * ((H + wm - 1) / wm) * ((W + wm - 1) / wm);
                const double px = (double)N * H * W;
                const mdx_conv_record rs[3] = {
                    {MDX_CONV_KERNEL_WINO_IN, 1, T, cw.cin, A * A, 4.0 * (px + (double)A * A * T) * cw.cin, 0.0, 0, 0},
                    {probe.gemm_kernel, 1, A * A * T, cw.cout, cw.cin, 2.0 * (double)A * A * T * cw.cout * cw.cin, 0.0,
                     0, 0},
                    {MDX_CONV_KERNEL_WINO_OUT, 1, T, cw.cout, A * A, 4.0 * ((double)A * A * T + px) * cw.cout, 0.0, 0,
                     0}};
                for (int q = 0; q < 3; ++q) {
                    c.prof.emplace_back();
                    ProfEv &p = c.prof.back();
                    p.e0 = probe.ev[2 * q];
                    p.e1 = probe.ev[2 * q + 1];
                    p.r = rs[q];
                }
            }
        } else {
            mdx::x3_weight_planes(cw.wp);  // split-plane mode: the pre-split weights
            chk(mdx_conv2d_splitk(x, N, H, W, cw.cin, cw.w, cw.b, cw.cout, cw.k, cw.k, cw.stride, cw.pad, residual,
                                  relu ? 1 : 0, out_mode, cw.dt, out_f32 ? 0 : cw.dt, out, 0, splitk, SPLITK_WS, s));
            mdx::x3_weight_planes(nullptr);
        }
        if (pe) {
            (void)hipEventRecord(pe->e1, s);
            int kid = -1, ks = 0;
            mdx_conv2d_last_plan(&kid, &ks);
            const int64_t M = (int64_t)N * OH * OW, K = (int64_t)cw.k * cw.k * cw.cin;
            pe->r = mdx_conv_record{kid + (out_f32 && cw.dt == 1 ? 10 : 0), ks, M, cw.cout, K,
                                    2.0 * (double)M * cw.cout * (cw.kalg ? cw.kalg : K), 0.0, cw.dt, 0};
        }
        return out;
    }
    // conv3 over x (N,H,W,Cin3) + the projection shortcut over x2 (N,H2,W2,Cin_sc), one GEMM
    void *conv3_shortcut(const void *x, int N, int H, int W, const void *x2, int H2, int W2, const ConvW &cw) {
        void *out = alloc((size_t)N * H * W * cw.cout * m.es);
        if (c.dry || !ok()) return out;
        ProfEv *pe = nullptr;
        if (m.profile) {
            c.prof.emplace_back();
            pe = &c.prof.back();
            (void)hipEventCreate(&pe->e0);
            (void)hipEventCreate(&pe->e1);
            (void)hipEventRecord(pe->e0, s);
        }
        chk(mdx_conv2d_dual(x, N, H, W, cw.cin, x2, H2, W2, cw.kalg, cw.stride, cw.w, cw.b, cw.cout, 1, m.dt, out,
                            splitk, SPLITK_WS, s));
        if (pe) {
            (void)hipEventRecord(pe->e1, s);
            int kid = -1, ks = 0;
            mdx_conv2d_last_plan(&kid, &ks);
            const int64_t M = (int64_t)N * H * W, K = (int64_t)cw.cin + cw.kalg;
            pe->r = mdx_conv_record{kid, ks, M, cw.cout, K, 2.0 * (double)M * cw.cout * K, 0.0, m.dt, 0};
        }
        return out;
    }
    void *last_gn_ws = nullptr;
    size_t last_gn_ws_bytes = 0;
    void *groupnorm(const void *x, int N, int H, int W, const GnW &g, const void *up, int fuse) {
        const int C = m.cfg.fpn_out_channels, G = m.cfg.gn_groups;
        void *out = alloc((size_t)N * H * W * C * m.es);
        last_gn_ws_bytes = (size_t)mdx_groupnorm_workspace_bytes(N, H, W, G);
        void *ws = alloc(last_gn_ws_bytes);
        last_gn_ws = ws;
        if (!c.dry && ok())
            chk(mdx_groupnorm(x, N, H, W, C, G, m.cfg.gn_eps, g.g, g.b, up, fuse, m.dt, out, (float *)ws, s));
        return out;
    }
    // planes: fp32 pooled rows written as bf16 planes (mdx_roi_align dtype 2)
    // out_dt: dtype of the pooled rows (the heads' dtype); pooled in the
    // trunk's dtype and converted when they differ (mixed configuration)
    void *roi_align(void *const *feats, const int *fh, const int *fw, const float *rois, const int *counts, int R,
                    int per_image, int P, bool planes = false, int out_dt = -1) {
        const int C = m.cfg.fpn_out_channels;
        if (out_dt >= 0 && out_dt != m.dt && !planes) {
            void *pooled = roi_align(feats, fh, fw, rois, counts, R, per_image, P);
            void *cvt = alloc((size_t)R * P * P * C * (out_dt == 1 ? 2 : 4));
            if (!c.dry && ok()) chk(mdx_convert(pooled, (int64_t)R * P * P * C, m.dt, cvt, out_dt, s));
            return cvt;
        }
        void *out = alloc(planes ? (size_t)mdx_x6_plane_bytes(R, P * P * C) : (size_t)R * P * P * C * m.es);
        // the box pooler (per_image = post-NMS proposals) runs in level/band order
        int *order = per_image >= 256 ? (int *)alloc((size_t)R * sizeof(int)) : nullptr;
        const float sc[4] = {1.f / 4, 1.f / 8, 1.f / 16, 1.f / 32};
        if (!c.dry && ok())
            chk(mdx_roi_align_ex((const void *const *)feats, fh, fw, sc, 4, 2, C, rois, counts, R, per_image, P,
                                 m.cfg.pooler_sampling_ratio, m.cfg.pooler_aligned, m.cfg.canonical_box_size,
                                 m.cfg.canonical_level, planes ? 2 : m.dt, order, out, s));
        return out;
    }

    void run(const uint8_t *frames, int B, int h, int w, const uint8_t *lut, const mdx_model_outputs *o) {
        const mdx_model_cfg &cfg = m.cfg;
        const int d = cfg.size_divisibility;
        const int Hp = (h + d - 1) / d * d, Wp = (w + d - 1) / d * d;
        const int D = cfg.detections_per_image, C = cfg.fpn_out_channels;
        splitk = alloc(SPLITK_WS);
        // preprocess (+ scale LUT), space-to-depth for the stem
        const int Hs = Hp / 2 + 1, Ws = Wp / 2 + 1;
        const int s2c = m.stem_fold ? 8 : 16;
        void *x = alloc((size_t)B * Hs * Ws * s2c * m.es);
        uint8_t ident[256];
        for (int i = 0; i < 256; ++i) ident[i] = (uint8_t)i;
        if (!c.dry && ok()) {
            if (m.stem_fold)
                chk(mdx_preprocess_s2d_folded(frames, B, h, w, lut ? lut : ident, Hp, Wp, m.dt, x, s));
            else
                chk(mdx_preprocess_s2d(frames, B, h, w, lut ? lut : ident, cfg.pixel_mean, cfg.pixel_std,
                                       cfg.in_channels, Hp, Wp, m.dt, x, s));
        }
        name("input_s2d", x, B, Hs, Ws, s2c, m.dt);
        // backbone
        int H, W;
        void *y = conv(x, B, Hs, Ws, m.stem, true, H, W);
        const int PH = (H + 2 - 3) / 2 + 1, PW = (W + 2 - 3) / 2 + 1;
        void *xp = alloc((size_t)B * PH * PW * m.stem.cout * m.es);
        if (!c.dry && ok()) chk(mdx_maxpool2d(y, B, H, W, m.stem.cout, 3, 2, 1, m.dt, xp, s));
        H = PH;
        W = PW;
        void *res[4] = {};
        int rh[4] = {}, rw[4] = {}, rc_[4] = {};
        void *cur = xp;
        for (const Block &blk : m.blocks) {
            int h1, w1, h2, w2, h3, w3;
            const void *sc = cur;
            // (the split-plane mode runs every conv on its own kernels)
            const bool fused = blk.c3sc.w && pol().fp32_split == 0;
            if (blk.has_sc && !fused) sc = conv(cur, B, H, W, blk.sc, false, h1, w1);
            void *t1 = conv(cur, B, H, W, blk.c1, true, h1, w1);
            void *t2 = conv(t1, B, h1, w1, blk.c2, true, h2, w2);
            if (fused) {
                cur = conv3_shortcut(t2, B, h2, w2, cur, H, W, blk.c3sc);
                h3 = h2;
                w3 = w2;
            } else
                cur = conv(t2, B, h2, w2, blk.c3, true, h3, w3, sc);
            H = h3;
            W = w3;
            res[blk.stage] = cur;
            rh[blk.stage] = H;
            rw[blk.stage] = W;
            rc_[blk.stage] = blk.c3.cout;
        }
        static const char *rn[4] = {"res2", "res3", "res4", "res5"};
        for (int i = 0; i < 4; ++i) name(rn[i], res[i], B, rh[i], rw[i], rc_[i], m.dt);
        // FPN, coarse to fine: lateral 1x1 + GN (fused nearest-x2 top-down add / avg), output 3x3 + GN
        void *feat[5] = {};
        int fh[5], fw[5];
        const void *prev = nullptr;
        const int fuse = cfg.fpn_fuse_avg ? 2 : 1;
        for (int i = 3; i >= 0; --i) {
            int oh, ow;
            void *lat = conv(res[i], B, rh[i], rw[i], m.fpn_lat[i], false, oh, ow);
            void *pv = groupnorm(lat, B, rh[i], rw[i], m.gn_lat[i], prev, prev ? fuse : 0);
            prev = pv;
            static const bool shadow_ws = getenv("MDX_DEBUG_SHADOW") != nullptr;
            if (shadow_ws && i == 3) {
                void *a0 = alloc(last_gn_ws_bytes);
                if (!c.dry && ok()) (void)hipMemcpyAsync(a0, last_gn_ws, last_gn_ws_bytes, hipMemcpyDeviceToDevice, s);
                name("shadow_gnws5", a0, 1, 1, 1, (int64_t)last_gn_ws_bytes / 4, 0);
                name("gnws5", last_gn_ws, 1, 1, 1, (int64_t)last_gn_ws_bytes / 4, 0);
            }
            void *o = conv(pv, B, rh[i], rw[i], m.fpn_out[i], false, oh, ow);
            feat[i] = groupnorm(o, B, rh[i], rw[i], m.gn_out[i], nullptr, 0);
            static const char *ln[4] = {"fpn_lateral2", "fpn_lateral3", "fpn_lateral4", "fpn_lateral5"};
            static const char *gn[4] = {"fpn_inner2", "fpn_inner3", "fpn_inner4", "fpn_inner5"};
            static const char *on[4] = {"fpn_output2", "fpn_output3", "fpn_output4", "fpn_output5"};
            name(ln[i], lat, B, rh[i], rw[i], C, m.dt);
            name(gn[i], pv, B, rh[i], rw[i], C, m.dt);
            name(on[i], o, B, rh[i], rw[i], C, m.dt);
            static const bool shadow = getenv("MDX_DEBUG_SHADOW") != nullptr;
            if (shadow) {  // debugging aid: copies of the GN outputs taken right after they are written
                static const char *sg[4] = {"shadow_inner2", "shadow_inner3", "shadow_inner4", "shadow_inner5"};
                static const char *sp[4] = {"shadow_p2", "shadow_p3", "shadow_p4", "shadow_p5"};
                const size_t nb = (size_t)B * rh[i] * rw[i] * C * m.es;
                void *a1 = alloc(nb), *a2 = alloc(nb);
                if (!c.dry && ok()) {
                    (void)hipMemcpyAsync(a1, pv, nb, hipMemcpyDeviceToDevice, s);
                    (void)hipMemcpyAsync(a2, feat[i], nb, hipMemcpyDeviceToDevice, s);
                }
                name(sg[i], a1, B, rh[i], rw[i], C, m.dt);
                name(sp[i], a2, B, rh[i], rw[i], C, m.dt);
            }
            fh[i] = rh[i];
            fw[i] = rw[i];
        }
        fh[4] = (fh[3] - 1) / 2 + 1;
        fw[4] = (fw[3] - 1) / 2 + 1;
        feat[4] = alloc((size_t)B * fh[4] * fw[4] * C * m.es);
        if (!c.dry && ok()) chk(mdx_maxpool2d(feat[3], B, fh[3], fw[3], C, 1, 2, 0, m.dt, feat[4], s));
        static const char *pn[5] = {"p2", "p3", "p4", "p5", "p6"};
        for (int i = 0; i < 5; ++i) name(pn[i], feat[i], B, fh[i], fw[i], C, m.dt);
        // RPN
        const float *heads[5];
        int strides[5];
        for (int l = 0; l < 5; ++l) {
            int oh, ow;
            void *t = conv(feat[l], B, fh[l], fw[l], m.rpn_conv, true, oh, ow);
            heads[l] = (const float *)conv(t, B, fh[l], fw[l], m.rpn_head, false, oh, ow, nullptr, true);
            strides[l] = 4 << l;
        }
        const int post = cfg.rpn_post_nms_topk;
        float *props = (float *)alloc((size_t)B * post * 4 * 4);
        float *pscores = (float *)alloc((size_t)B * post * 4);
        int *pcount = (int *)alloc((size_t)B * 4);
        void *rws = alloc((size_t)mdx_rpn_workspace_bytes(B, 5, cfg.rpn_pre_nms_topk));
        if (!c.dry && ok())
            chk(mdx_rpn_proposals(heads, fh, fw, strides, 5, B, cfg.n_aspect_ratios, m.cell_anchors.data(),
                                  cfg.anchor_offset, h, w, cfg.rpn_pre_nms_topk, post, cfg.rpn_nms_thresh,
                                  cfg.rpn_min_box_size, (float)std::log(1000.0 / 16), cfg.rpn_bbox_reg_weights, props,
                                  pscores, pcount, rws, s));
        name("proposals", props, B, post, 4, 1, 0);
        name("proposal_scores", pscores, B, post, 1, 1, 0);
        name("proposal_count", pcount, B, 1, 1, 1, 2);
        // box head + fast_rcnn_inference
        const int R = cfg.box_pooler_resolution;
        // split-plane mode: the pooler writes fc1's A operand as bf16 planes
        const bool pl = m.dt == 0 && !m.fc.empty() && m.fc[0].x6 && pol().fp32_split == 6 &&
                        (pol().roi_mode == 4 || pol().roi_mode == 5) && (R * R * C) % 16 == 0;
        void *pooled = roi_align(feat, fh, fw, props, pcount, B * post, post, R, pl);
        if (pl)
            name("box_pooled", pooled, (int64_t)B * post, R * R * C / 16, 3, 16, 3);
        else
            name("box_pooled", pooled, (int64_t)B * post, R, R, C, m.dt);
        const void *yv = pooled;
        int oh, ow;
        for (size_t i = 0; i < m.fc.size(); ++i)
            yv = conv(yv, B * post, 1, 1, m.fc[i], true, oh, ow, nullptr, false, 0, nullptr, pl && i == 0);
        float *pred = (float *)conv(yv, B * post, 1, 1, m.box_pred, false, oh, ow, nullptr, true);
        name("box_pred", pred, (int64_t)B * post, m.box_pred.cout, 1, 1, 0);
        if (!c.dry && ok())
            chk(mdx_box_postprocess(pred, m.box_pred.cout, props, pcount, B, post, D, cfg.score_thresh,
                                    cfg.nms_thresh, h, w, cfg.box_reg_weights, (float)std::log(1000.0 / 16),
                                    o->boxes, o->scores, o->classes, o->ndet, s));
        const int R2 = B * D;
        if (cfg.mask_on) {
            const int M = cfg.mask_pooler_resolution;
            const void *t = roi_align(feat, fh, fw, o ? o->boxes : nullptr, o ? o->ndet : nullptr, R2, D, M, false, m.hdt);
            for (const ConvW &cw : m.mask_convs) t = conv(t, R2, M, M, cw, true, oh, ow);
            t = conv(t, R2, M, M, m.mask_deconv, true, oh, ow, nullptr, false, 1);
            float *logits = (float *)conv(t, R2, 2 * M, 2 * M, m.mask_pred, false, oh, ow, nullptr, true);
            name("mask_logits", logits, R2, 2 * M, 2 * M, 1, 0);
            if (!c.dry && ok() && o->masks)
                chk(mdx_paste_masks(logits, o->boxes, o->ndet, B, D, 2 * M, h, w, o->mask_plane_stride,
                                    cfg.mask_threshold, o->masks, s));
        }
        if (cfg.keypoint_on) {
            const int Pk = cfg.keypoint_pooler_resolution, K = cfg.num_keypoints;
            const void *t = roi_align(feat, fh, fw, o ? o->boxes : nullptr, o ? o->ndet : nullptr, R2, D, Pk, false, m.hdt);
            for (const ConvW &cw : m.kp_convs) t = conv(t, R2, Pk, Pk, cw, true, oh, ow);
            float *yk = (float *)conv(t, R2, Pk, Pk, m.kp_deconv, false, oh, ow, nullptr, true);
            float *low = (float *)alloc((size_t)R2 * K * 4 * Pk * Pk * 4);
            float *hm = o && o->keypoint_heatmaps ? o->keypoint_heatmaps
                                                  : (float *)alloc((size_t)R2 * K * 16 * Pk * Pk * 4);
            if (!c.dry && ok()) {
                chk(mdx_deconv_col2im(yk, m.kp_deconv_b, R2, Pk, Pk, K, low, s));
                chk(mdx_upsample_bilinear2x(low, R2 * K, 2 * Pk, 2 * Pk, hm, s));
                if (o->keypoints)
                    chk(mdx_heatmaps_to_keypoints(hm, o->boxes, o->ndet, B, D, K, 4 * Pk, o->keypoints, s));
            }
            name("keypoint_heatmaps", hm, R2, K, 4 * Pk, 4 * Pk, 0);
        }
    }
};

Ctx *get_ctx(Model &m, hipStream_t s) {
    std::lock_guard<std::mutex> g(m.mu);
    auto &p = m.ctx[s];
    if (!p) p.reset(new Ctx());
    return p.get();
}

int reserve(Model &m, Ctx &c, int B, int h, int w, hipStream_t s) {
    c.dry = true;
    c.off = 0;
    c.wino_need = 0;
    Fwd f{m, c, s};
    f.run(nullptr, B, h, w, nullptr, nullptr);
    c.dry = false;
    if (c.wino_need > c.wino_cap) {
        if (c.wino_base) {
            MDX_HIP(hipStreamSynchronize(s));
            MDX_HIP(hipFree(c.wino_base));
            c.wino_base = nullptr;
            c.wino_cap = 0;
        }
        if (hipMalloc((void **)&c.wino_base, c.wino_need) != hipSuccess) {
            (void)hipGetLastError();
            set_error("mdx_model_reserve: cannot allocate a %.1f GB Winograd workspace", c.wino_need / 1e9);
            return MDX_ENOMEM;
        }
        c.wino_cap = c.wino_need;
    }
    const size_t need = c.off + 4096;
    if (need <= c.cap) return MDX_OK;
    if (c.base) {
        MDX_HIP(hipStreamSynchronize(s));  // the old arena may still be read by queued work
        MDX_HIP(hipFree(c.base));
        c.base = nullptr;
        c.cap = 0;
    }
    if (hipMalloc((void **)&c.base, need) != hipSuccess) {
        (void)hipGetLastError();
        set_error("mdx_model_reserve: cannot allocate a %.1f GB workspace", need / 1e9);
        return MDX_ENOMEM;
    }
    c.cap = need;
    return MDX_OK;
}

}  // namespace
}  // namespace mdx

using namespace mdx;

// mdx_policy.stem_fold: fp32 handles fold the stem to the 2-channel (value,
// inside) form (1, default) or keep the normalised 3-channel input (0).
// mdx_policy.fuse_shortcut: 0 off, 1 fp32 handles (default: fp32 loop
// +1.2 %), 2 fp32 and fp16 handles (fp16 R50 B=32 +2.5 %, R101 B=64 +0.8 %,
// but the full-frame fp16 case then passes the detection check on 25 of 32
// frames, one under its 80 % bar).  Both are read at mdx_model_create.
extern "C" int mdx_model_create(const void *blob, int64_t blob_bytes, const mdx_model_cfg *cfg, int device,
                                mdx_model_t *out) {
    MDX_REQUIRE(blob && cfg && out && blob_bytes >= 12, "mdx_model_create: null argument or blob shorter than its header");
    *out = nullptr;
    MDX_REQUIRE(cfg->depth == 50 || cfg->depth == 101, "mdx_model_create: depth must be 50 or 101");
    MDX_REQUIRE(cfg->dtype == 0 || cfg->dtype == 1, "mdx_model_create: dtype must be 0 (f32) or 1 (f16)");
    MDX_REQUIRE(cfg->head_dtype == 0 || cfg->head_dtype == 1,
                "mdx_model_create: head_dtype must be 0 (as dtype) or 1 (f16 mask + keypoint heads)");
    MDX_REQUIRE(cfg->num_classes == 1, "mdx_model_create: the extraction model has one class (NUM_CLASSES=1)");
    MDX_REQUIRE(cfg->n_anchor_sizes == 5 && cfg->n_aspect_ratios >= 1 && cfg->n_aspect_ratios <= 8,
                "mdx_model_create: 5 anchor sizes (one per level p2..p6) and 1..8 aspect ratios");
    MDX_REQUIRE(cfg->rpn_bbox_reg_weights[0] > 0.f && cfg->rpn_bbox_reg_weights[1] > 0.f &&
                    cfg->rpn_bbox_reg_weights[2] > 0.f && cfg->rpn_bbox_reg_weights[3] > 0.f &&
                    cfg->box_reg_weights[0] > 0.f && cfg->box_reg_weights[1] > 0.f && cfg->box_reg_weights[2] > 0.f &&
                    cfg->box_reg_weights[3] > 0.f,
                "mdx_model_create: box regression weights must be positive");
    MDX_REQUIRE(cfg->fpn_out_channels % 8 == 0 && cfg->gn_groups > 0 && cfg->detections_per_image >= 1 &&
                    cfg->detections_per_image <= 16 && cfg->n_keypoint_convs >= 0 && cfg->n_keypoint_convs <= 16 &&
                    cfg->in_channels >= 1 && cfg->in_channels <= 3 && cfg->size_divisibility >= 2 &&
                    cfg->size_divisibility % 2 == 0,
                "mdx_model_create: unsupported configuration");
    std::unordered_map<std::string, HostT> sd;
    if (!parse_blob(blob, blob_bytes, sd)) return MDX_EINVAL;
    MDX_HIP(hipSetDevice(device));
    std::unique_ptr<Model> m(new Model());
    m->cfg = *cfg;
    m->dev = device;
    m->dt = cfg->dtype;
    m->hdt = cfg->head_dtype == 1 ? 1 : cfg->dtype;
    m->es = cfg->dtype == 1 ? 2 : 4;
    m->policy = pol();
    PolicyScope ps(&m->policy);
    m->stem_fold = cfg->dtype == 0 && m->policy.stem_fold;
    m->fuse_sc = m->policy.fuse_shortcut == 2 || (m->policy.fuse_shortcut == 1 && cfg->dtype == 0);
    std::string err;
    if (!pack(*m, sd, err)) {
        set_error("mdx_model_create: %s", err.c_str());
        return MDX_EINVAL;
    }
    *out = m.release();
    return MDX_OK;
}

extern "C" int mdx_model_get_policy(mdx_model_t model, mdx_policy *out) {
    MDX_REQUIRE(model && out, "mdx_model_get_policy: null argument");
    *out = ((Model *)model)->policy;
    return MDX_OK;
}

extern "C" int mdx_model_destroy(mdx_model_t model) {
    if (model) {
        Model *m = (Model *)model;
        for (auto &kv : m->ctx) (void)hipStreamSynchronize(kv.first);
        delete m;
    }
    return MDX_OK;
}

extern "C" int mdx_model_reserve(mdx_model_t model, int B, int h, int w, mdx_stream_t stream) {
    MDX_REQUIRE(model && B > 0 && h > 0 && w > 0, "mdx_model_reserve: bad arguments");
    Model &m = *(Model *)model;
    PolicyScope ps(&m.policy);
    hipStream_t s = as_stream(stream);
    return reserve(m, *get_ctx(m, s), B, h, w, s);
}

extern "C" int mdx_model_forward(mdx_model_t model, const uint8_t *frames, int B, int h, int w, const uint8_t *lut,
                                 const mdx_model_outputs *out, mdx_stream_t stream) {
    MDX_REQUIRE(model && frames && out && out->boxes && out->scores && out->classes && out->ndet,
                "mdx_model_forward: null argument");
    MDX_REQUIRE(B > 0 && h > 0 && w > 0, "mdx_model_forward: empty batch");
    Model &m = *(Model *)model;
    MDX_REQUIRE(!out->masks || out->mask_plane_stride >= (int64_t)h * w,
                "mdx_model_forward: mask_plane_stride < h*w");
    hipStream_t s = as_stream(stream);
    PolicyScope ps(&m.policy);
    Ctx &c = *get_ctx(m, s);
    const int r = reserve(m, c, B, h, w, s);
    if (r != MDX_OK) return r;
    for (auto &p : c.prof) {
        (void)hipEventDestroy(p.e0);
        (void)hipEventDestroy(p.e1);
    }
    c.prof.clear();
    c.named.clear();
    c.off = 0;
    Fwd f{m, c, s};
    f.run(frames, B, h, w, lut, out);
    return f.rc;
}

extern "C" int mdx_model_tensor_info(mdx_model_t model, mdx_stream_t stream, const char *name, int64_t shape[4],
                                     int *dtype) {
    MDX_REQUIRE(model && name && shape && dtype, "mdx_model_tensor_info: null argument");
    Model &m = *(Model *)model;
    Ctx &c = *get_ctx(m, as_stream(stream));
    auto it = c.named.find(name);
    MDX_REQUIRE(it != c.named.end(), "mdx_model_tensor_info: no intermediate \"%s\" on this stream", name);
    for (int i = 0; i < 4; ++i) shape[i] = it->second.shape[i];
    *dtype = it->second.dtype;
    return MDX_OK;
}

extern "C" int mdx_model_tensor_copy(mdx_model_t model, mdx_stream_t stream, const char *name, void *dst,
                                     int64_t bytes) {
    MDX_REQUIRE(model && name && dst && bytes >= 0, "mdx_model_tensor_copy: null argument");
    Model &m = *(Model *)model;
    hipStream_t s = as_stream(stream);
    Ctx &c = *get_ctx(m, s);
    auto it = c.named.find(name);
    MDX_REQUIRE(it != c.named.end(), "mdx_model_tensor_copy: no intermediate \"%s\" on this stream", name);
    const TensorRec &t = it->second;
    const int64_t have = t.shape[0] * t.shape[1] * t.shape[2] * t.shape[3] * (t.dtype == 1 || t.dtype == 3 ? 2 : 4);
    MDX_REQUIRE(bytes <= have, "mdx_model_tensor_copy: %lld bytes requested, \"%s\" has %lld", (long long)bytes,
                name, (long long)have);
    MDX_HIP(hipMemcpyAsync(dst, t.p, (size_t)bytes, hipMemcpyDeviceToDevice, s));
    return MDX_OK;
}

extern "C" int mdx_model_debug_fill(mdx_model_t model, int B, int h, int w, int byte, mdx_stream_t stream) {
    MDX_REQUIRE(model && byte >= 0 && byte <= 255, "mdx_model_debug_fill: bad arguments");
    Model &m = *(Model *)model;
    hipStream_t s = as_stream(stream);
    PolicyScope ps(&m.policy);
    Ctx &c = *get_ctx(m, s);
    const int r = reserve(m, c, B, h, w, s);
    if (r != MDX_OK) return r;
    MDX_HIP(hipMemsetAsync(c.base, byte, c.cap, s));
    return MDX_OK;
}

extern "C" int mdx_model_debug_arena(mdx_model_t model, mdx_stream_t stream, const char *name, int64_t *offset,
                                     int64_t *arena_bytes, void *dst, int64_t dst_bytes) {
    MDX_REQUIRE(model, "mdx_model_debug_arena: null model");
    Model &m = *(Model *)model;
    hipStream_t s = as_stream(stream);
    Ctx &c = *get_ctx(m, s);
    if (arena_bytes) *arena_bytes = (int64_t)c.cap;
    if (name && offset) {
        auto it = c.named.find(name);
        MDX_REQUIRE(it != c.named.end(), "mdx_model_debug_arena: no intermediate \"%s\"", name);
        *offset = it->second.offset;
    }
    if (dst) {
        MDX_REQUIRE(dst_bytes >= 0 && (size_t)dst_bytes <= c.cap, "mdx_model_debug_arena: bad copy size");
        MDX_HIP(hipMemcpyAsync(dst, c.base, (size_t)dst_bytes, hipMemcpyDeviceToDevice, s));
    }
    return MDX_OK;
}

extern "C" int mdx_model_profile(mdx_model_t model, int on) {
    MDX_REQUIRE(model, "mdx_model_profile: null model");
    Model &m = *(Model *)model;
    const int old = m.profile ? 1 : 0;
    m.profile = on != 0;
    return old;
}

extern "C" int mdx_model_profile_read(mdx_model_t model, mdx_conv_record *out, int max) {
    MDX_REQUIRE(model && (out || max == 0), "mdx_model_profile_read: null argument");
    Model &m = *(Model *)model;
    std::lock_guard<std::mutex> g(m.mu);
    int n = 0;
    for (auto &kv : m.ctx)
        for (auto &p : kv.second->prof) {
            float ms = 0.f;
            if (hipEventElapsedTime(&ms, p.e0, p.e1) != hipSuccess) {
                (void)hipGetLastError();
                ms = -1.f;
            }
            if (n < max) {
                out[n] = p.r;
                out[n].ms = ms;
            }
            ++n;
        }
    return n < max ? n : max;
}
