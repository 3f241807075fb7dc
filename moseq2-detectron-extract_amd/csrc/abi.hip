// Error state, version and kernel-selection policy of the mdx C ABI.
#include "common.h"

namespace mdx {
static thread_local std::string g_err;
void set_error(const char *fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
}

static mdx_policy library_defaults() {
    mdx_policy p{};
    p.winograd = 6;
    p.winograd_min_cin = 64;
    p.winograd_dma = 0;
    p.winograd_dma_min_wgs = 384;
    p.wino_slice_mb = 0;
    p.fp32_split = 0;
    p.x3_narrow = 1;
    p.x3_single_stage = 1;
    p.large_tiles = 1;
    p.dma128 = 0;
    p.dma128_min_tiles = 1536;
    p.dma128_interleave = 1;
    p.dma_f32 = 0;
    p.pointwise = 1;
    p.single_stage = 4;
    p.direct_epilogue = 1;
    p.narrow_kmax = 128;
    p.head_f32 = 1;
    p.stream1x1 = 1;
    p.stream1x1_min_m = 65536;
    p.stem_fold = 1;
    p.fuse_shortcut = 1;
    p.rpn_sliced = 1;
    p.roi_mode = 4;
    p.roi_xcd_order = 1;
    p.roi_sorted = 1;
    p.f16_pingpong = 1;
    return p;
}
// the calling thread's policy, and the model handle's while one of its entry
// points runs on this thread (PolicyScope)
static thread_local mdx_policy t_thread = library_defaults();
static thread_local const mdx_policy *t_active = nullptr;
const mdx_policy &pol() { return t_active ? *t_active : t_thread; }
PolicyScope::PolicyScope(const mdx_policy *p) : prev(t_active) { t_active = p; }
PolicyScope::~PolicyScope() { t_active = prev; }
}  // namespace mdx

extern "C" const char *mdx_last_error(void) { return mdx::g_err.c_str(); }
extern "C" const char *mdx_version(void) { return "mdx 0.2.0 gfx950"; }

extern "C" int mdx_policy_defaults(mdx_policy *out) {
    MDX_REQUIRE(out, "mdx_policy_defaults: null pointer");
    *out = mdx::library_defaults();
    return MDX_OK;
}
extern "C" int mdx_policy_get(mdx_policy *out) {
    MDX_REQUIRE(out, "mdx_policy_get: null pointer");
    *out = mdx::pol();
    return MDX_OK;
}
extern "C" int mdx_policy_set(const mdx_policy *p) {
    MDX_REQUIRE(p, "mdx_policy_set: null pointer");
    MDX_REQUIRE(p->winograd == 0 || p->winograd == 2 || p->winograd == 4 || p->winograd == 6,
                "mdx_policy_set: winograd must be 0, 2, 4 or 6 (got %d)", p->winograd);
    MDX_REQUIRE(p->fp32_split == 0 || p->fp32_split == 6 || p->fp32_split == 9,
                "mdx_policy_set: fp32_split must be 0, 6 or 9 (got %d)", p->fp32_split);
    MDX_REQUIRE(p->roi_mode >= 0 && p->roi_mode <= 7, "mdx_policy_set: roi_mode must be 0-7 (got %d)", p->roi_mode);
    MDX_REQUIRE(p->single_stage >= 0 && p->single_stage <= 4, "mdx_policy_set: single_stage must be 0-4");
    MDX_REQUIRE(p->winograd_min_cin >= 0 && p->narrow_kmax >= 0 && p->wino_slice_mb >= 0 &&
                    p->dma128_min_tiles >= 0 && p->winograd_dma_min_wgs >= 0 && p->stream1x1_min_m >= 0,
                "mdx_policy_set: thresholds must be >= 0");
    mdx::t_thread = *p;
    return MDX_OK;
}
