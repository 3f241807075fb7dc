// Host-side (CPU) instance tracker of ProcessFeaturesStep.__select_instances
// (M/pipeline/process_features_step.py:35-38 tracker setup, :133-160 the
// selection): norfair 2.x Tracker(distance_function='euclidean',
// distance_threshold=50, initialization_delay=0, hit_counter_max=3) with the
// default OptimizedKalmanFilter (R=4, Q=0.1, pos_variance=10,
// pos_vel_covariance=0, vel_variance=1) over 1-point detections.  The state
// carries across chunks behind a handle; one call per chunk, no GIL.  Same
// double arithmetic as instances.py's statement of the algorithm (float32
// distance matrix, greedy matching in ascending (distance, detection, object)
// order), so decisions are identical; checked against oracle/norfair_ref.py.
#include <algorithm>
#include <cmath>
#include <vector>

#include "common.h"

#pragma clang fp contract(off)

namespace {

constexpr double DIST_THR = 50.0, KF_R = 4.0, KF_Q = 0.1;
constexpr int HIT_MAX = 3, POINT_HIT_MAX = 4;

struct Obj {
    double pos[2], vel[2];
    double p, pv, vv;
    int hit_counter, point_hit;
    long long age;
    long long last_frame;
    int last_slot;
};

struct Tracker {
    int expected;
    std::vector<Obj> objs;
};

void hit(Obj &o, const double *pt, long long g, int s) {
    o.last_frame = g;
    o.last_slot = s;
    o.hit_counter = std::min(o.hit_counter + 2, HIT_MAX);
    o.point_hit = std::min(std::max(o.point_hit + 2, 0), POINT_HIT_MAX);
    const double vpp = o.pv + o.vv;
    const double added = o.p + o.pv + vpp + KF_Q + KF_R;
    const double r_over = KF_R / added, v_over = vpp / added;
    for (int c = 0; c < 2; ++c) {
        const double err = pt[c] - o.pos[c];
        o.pos[c] += (1.0 - r_over) * err;
        o.vel[c] += v_over * err;
    }
    o.p = (1.0 - r_over) * KF_R;
    o.pv = v_over * KF_R;
    o.vv += KF_Q - (v_over * v_over) * added;
}

// Tracker.update: returns false on a NaN distance (the reference raises)
bool update(Tracker &t, const double *pts, int nd, long long g, std::vector<int> &active) {
    std::vector<Obj> alive;
    alive.reserve(t.objs.size() + nd);
    for (const Obj &o : t.objs)
        if (o.hit_counter >= 0) alive.push_back(o);
    t.objs.swap(alive);
    for (Obj &o : t.objs) {
        o.hit_counter -= 1;
        o.point_hit -= 1;
        o.age += 1;
        o.pos[0] += o.vel[0];
        o.pos[1] += o.vel[1];
    }
    const int no = (int)t.objs.size();
    std::vector<char> matched(nd, 0);
    if (nd && no) {
        struct Cand {
            float d;
            int i, j;
        };
        std::vector<Cand> cand;
        cand.reserve((size_t)nd * no);
        for (int i = 0; i < nd; ++i)
            for (int j = 0; j < no; ++j) {
                const double dy = pts[2 * i] - t.objs[j].pos[0], dx = pts[2 * i + 1] - t.objs[j].pos[1];
                const float d = (float)std::sqrt(dy * dy + dx * dx);
                if (std::isnan(d)) return false;
                cand.push_back({d, i, j});
            }
        std::sort(cand.begin(), cand.end(), [](const Cand &a, const Cand &b) {
            if (a.d != b.d) return a.d < b.d;
            if (a.i != b.i) return a.i < b.i;
            return a.j < b.j;
        });
        std::vector<char> used_j(no, 0);
        for (const Cand &c : cand) {
            if (!((double)c.d < DIST_THR)) break;
            if (matched[c.i] || used_j[c.j]) continue;
            matched[c.i] = 1;
            used_j[c.j] = 1;
            hit(t.objs[c.j], pts + 2 * c.i, g, c.i);
        }
    }
    for (int i = 0; i < nd; ++i)
        if (!matched[i]) {
            Obj o;
            o.pos[0] = pts[2 * i];
            o.pos[1] = pts[2 * i + 1];
            o.vel[0] = o.vel[1] = 0.0;
            o.p = 10.0;
            o.pv = 0.0;
            o.vv = 1.0;
            o.hit_counter = 1;
            o.point_hit = 1;
            o.age = 0;
            o.last_frame = g;
            o.last_slot = i;
            t.objs.push_back(o);
        }
    active.clear();
    for (int k = 0; k < (int)t.objs.size(); ++k)
        if (t.objs[k].hit_counter >= 0) active.push_back(k);
    return true;
}

}  // namespace

extern "C" void *mdx_instance_tracker_create(int expected_instances) {
    if (expected_instances < 1) return nullptr;
    Tracker *t = new Tracker;
    t->expected = expected_instances;
    return t;
}

extern "C" int mdx_instance_tracker_destroy(void *handle) {
    delete static_cast<Tracker *>(handle);
    return MDX_OK;
}

extern "C" int mdx_instance_tracker_select(void *handle, const int *nkeep, const double *centers, int64_t n, int D,
                                           int64_t frame0, int *out_n, int64_t *out_ids) {
    MDX_REQUIRE(handle && (n == 0 || (nkeep && centers && out_n && out_ids)),
                "mdx_instance_tracker_select: null pointer");
    MDX_REQUIRE(D >= 1, "mdx_instance_tracker_select: D < 1");
    Tracker &t = *static_cast<Tracker *>(handle);
    const int E = t.expected;
    std::vector<int> active, live;
    for (int64_t f = 0; f < n; ++f) {
        const int k = nkeep[f];
        MDX_REQUIRE(k >= 0 && k <= D, "mdx_instance_tracker_select: nkeep[%lld] out of range", (long long)f);
        const long long g = frame0 + f;
        MDX_REQUIRE(update(t, centers + f * D * 2, k, g, active),
                    "mdx_instance_tracker_select: NaN distance at frame %lld", g);
        int64_t *ids = out_ids + f * E * 2;
        out_n[f] = -1;
        if (active.size() <= 1) continue;
        live.clear();
        for (int a : active)
            if (t.objs[a].point_hit > 0) live.push_back(a);
        std::stable_sort(live.begin(), live.end(), [&](int a, int b) { return t.objs[a].age < t.objs[b].age; });
        int m = 0;
        while (m < E && !live.empty()) {
            const Obj &o = t.objs[live.back()];
            live.pop_back();
            ids[2 * m] = o.last_frame;
            ids[2 * m + 1] = o.last_slot;
            ++m;
        }
        // unchanged: the frame's own detections in their order
        bool same = m == k;
        for (int s = 0; same && s < m; ++s) same = ids[2 * s] == g && ids[2 * s + 1] == s;
        out_n[f] = same ? -1 : m;
    }
    return MDX_OK;
}
