// pyramid_plan.cpp -- host plan of the fused pyramid pass (pyramid.hip) and a
// CPU emulation of that kernel over the plan (debug ABI, CPU tests).
//
// ComputePyramid (ORBextractor.cpp:1123-1148) makes level l from level l-1
// with resize(INTER_LINEAR): output row y of level l reads source rows
// yofs[y] and yofs[y] + 1 (clamped) of level l-1.  The kernel runs one frame
// per block in ticks.  At tick k the producer wave(s) write level-0 chunk k+1
// (tk_t0 rows) into an LDS ring, and every level l >= 1 computes the rows
// whose two source rows were in LDS before tick k, i.e. level-0 chunks <= k or
// level-(l-1) rows computed at ticks < k.  So all levels advance in the same
// tick with one barrier per tick, and no level is ever read back from HBM:
// the pass reads level 0 once and writes levels 1..L-1 once.
//
// Everything frame-independent is fixed here: the rows each level computes
// per tick, the ring sizes (the most rows a level still needs plus what its
// producer writes in the same tick), every row's LDS slot and the per-thread
// assignment of (level, quad) columns.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <vector>

#include "host_common.h"
#include "orbgpu_internal.h"
#include "orbgpu_kernels.h"

namespace orbgpu {

namespace {

#ifndef ORBGPU_PYR_T0
#define ORBGPU_PYR_T0 8  // level-0 rows per chunk (per tick)
#endif
#ifndef ORBGPU_PYR_LANES
#define ORBGPU_PYR_LANES 576  // compute lanes the row-group split may use (9 waves + the tail wave + the producer: two blocks per CU)
#endif

inline int round_up(int v, int a) { return (v + a - 1) / a * a; }

}  // namespace

// LDS byte offset of row r of level l in its ring (level 0: chunk runs)
int slot_offset(const Geom& g, int l, int r) {
    const LevelGeom& v = g.lv[l];
    if (l == 0) return v.tk_ring + ((r / g.tk_t0) % g.tk_nc0) * g.tk_cstride0 + (r % g.tk_t0) * v.tk_pitch;
    return v.tk_ring + (r % v.tk_ring_rows) * v.tk_pitch;
}

int plan_pyramid(Geom& g, const std::vector<int2>& ytab, const std::vector<int4>& ptab, int max_batch, PyrPlan& plan) {
    const int L = g.nlevels;
    plan.tab.clear();
    plan.ent.clear();
    if (L < 2) return ORBGPU_OK;
    const int T0 = ORBGPU_PYR_T0;
    const int H0 = g.lv[0].h;
    g.tk_t0 = T0;
    g.tk_k0 = (H0 + T0 - 1) / T0;
    auto y0 = [&](int l, int y) { return ytab[(size_t)g.lv[l].ytab_offset + y].x & 0xFFFF; };
    auto y1 = [&](int l, int y) { return ytab[(size_t)g.lv[l].ytab_offset + y].x >> 16; };
    for (int l = 1; l < L; ++l)
        for (int y = 0; y < g.lv[l].h; ++y)
            if (y0(l, y) > y1(l, y) || (y > 0 && (y0(l, y) < y0(l, y - 1) || y1(l, y) < y1(l, y - 1))))
                return fail(ORBGPU_ERR_UNSUPPORTED, "resize row taps are not monotone");

    // --- tick schedule: p[k][l] = rows of level l computed before tick k
    // (level 0: rows in LDS at the start of tick k = chunks 0..k)
    auto avail0 = [&](int k) { return std::min((k + 1) * T0, H0); };
    std::vector<std::vector<int>> p(1, std::vector<int>(L, 0));
    p[0][0] = avail0(0);
    for (int k = 0;; ++k) {
        if (k > 100000) return fail(ORBGPU_ERR_UNSUPPORTED, "pyramid tick plan does not terminate");
        std::vector<int> nx(L, 0);
        nx[0] = avail0(k + 1);
        bool done = true;
        for (int l = 1; l < L; ++l) {
            const int src = l == 1 ? avail0(k) : p[k][l - 1];
            int n = p[k][l];
            while (n < g.lv[l].h && y1(l, n) < src) ++n;
            nx[l] = n;
            if (n < g.lv[l].h) done = false;
        }
        p.push_back(nx);
        if (done) break;
    }
    const int K = (int)p.size() - 1;  // ticks: level l computes rows [p[k][l], p[k+1][l]) at tick k
    g.tk_ticks = K;

    // --- ring sizes.  Levels >= 1: at tick k, level l-1 must still hold rows
    // [lo, hi) where lo = the first source row of level l's next uncomputed
    // row and hi = the rows of level l-1 that exist at the end of tick k.
    // Level 0 arrives by LDS-DMA in chunk runs: during tick k chunk k+1 lands
    // and chunk k+2 is in flight, so the runs must hold the chunks from lo's
    // up to chunk k+2.
    std::vector<int> C(L, 0);
    int NC = 3;
    for (int k = 0; k < K; ++k)
        for (int l = 1; l < L; ++l) {
            if (p[k][l] >= g.lv[l].h) continue;
            const int lo = y0(l, p[k][l]);
            if (l == 1) {
                NC = std::max(NC, k + 3 - lo / T0);
            } else {
                C[l - 1] = std::max(C[l - 1], p[k + 1][l - 1] - lo);
            }
        }
    NC = std::min(NC, g.tk_k0 + 2);
    C[0] = NC * T0;
    for (int l = 1; l + 1 < L; ++l) C[l] = std::min(std::max(C[l], 2), g.lv[l].h);

    // --- row groups per level (a level's rows of one tick split into G
    // contiguous runs, each on its own lanes).  A wave's tick costs its
    // longest lane's rows, so split the level with the most rows per lane
    // while the lanes fit the block (one entry per lane, the producer waves
    // beside them).
    const int v4p = (g.lv[0].w + 15) / 16, pwaves = (T0 * v4p + 511) / 512;
    const int lane_budget = std::min(ORBGPU_PYR_LANES, 1024 - 64 * pwaves);
    std::vector<int> G(L, 1), mx(L, 0), octs(L, 0), tailq(L, 0);
    for (int l = 1; l < L; ++l) {
        for (int k = 0; k < K; ++k) mx[l] = std::max(mx[l], p[k + 1][l] - p[k][l]);
        const int Q = (g.lv[l].w + 3) / 4;
        tailq[l] = g.lv[l].qmain < Q ? 1 : 0;
        octs[l] = (Q - tailq[l] + 1) / 2;  // regular octs (the column entries below)
    }
    auto lanes = [&]() {  // regular octs, then the tail octs from a wave boundary
        int n = 0, t = 0;
        for (int l = 1; l < L; ++l) {
            n += octs[l] * G[l];
            t += tailq[l];
        }
        return round_up(n, 64) + (t ? 64 : 0);
    };
    for (;;) {
        int worst = 1;
        for (int l = 2; l < L; ++l)
            if ((mx[l] + G[l] - 1) / G[l] > (mx[worst] + G[worst] - 1) / G[worst]) worst = l;
        const int cur = (mx[worst] + G[worst] - 1) / G[worst];
        if (cur <= 1) break;
        G[worst] += 1;
        if (round_up(lanes(), 64) > lane_budget || (mx[worst] + G[worst] - 1) / G[worst] == cur) {
            G[worst] -= 1;
            break;
        }
    }
    // The tail octs (one wave of their own, below) split their level's rows
    // as finely as that wave allows: about one row per lane per tick.
    std::vector<int> GT(L, 0);
    int nt = 0;
    for (int l = 1; l < L; ++l) nt += (GT[l] = tailq[l] ? std::max(1, mx[l]) : 0);
    while (nt > 64) {
        int big = 1;
        for (int l = 2; l < L; ++l)
            if (GT[l] > GT[big]) big = l;
        --GT[big];
        --nt;
    }
    // range slots per tick: level l's regular groups, then its tail groups
    std::vector<int> base_r(L, 0), base_t(L, 0);
    int slots = 0;
    for (int l = 1; l < L; ++l) {
        base_r[l] = slots;
        slots += G[l];
        base_t[l] = slots;
        slots += GT[l];
    }
    g.tk_groups = slots;
    g.tk_rs = slots + 1;  // + the empty range of idle lanes

    // --- producer: LDS-DMA pieces of 16 B (one per lane), at most 8 per lane
    const int v4 = (g.lv[0].w + 15) / 16, items = T0 * v4;
    g.tk_pwaves = (items + 511) / 512;
    g.tk_np = (items + 64 * g.tk_pwaves - 1) / (64 * g.tk_pwaves);
    g.tk_nc0 = NC;
    g.tk_cstride0 = 16 * 64 * g.tk_pwaves * g.tk_np;  // >= T0 rows at the level-0 pitch

    // --- LDS layout: 16 B pad | ring 0 | ring 1 | ... | ring L-2 | 16 B pad | sink | plan table.
    // Ring rows of levels >= 1 get an odd number of 16-byte units per row
    // (ORBGPU_PYR_STAGGER): consecutive rows then start 4, 12, 20 or 28
    // banks apart instead of on the same bank, so lanes of one instruction
    // that read different rows of a ring at nearby columns (different row
    // groups / levels in one wave) do not pile onto the same banks.  Level 0
    // keeps 16 * v4: its LDS-DMA pieces land contiguously.
#ifndef ORBGPU_PYR_STAGGER
#define ORBGPU_PYR_STAGGER 1
#endif
    int off = 16;
    for (int l = 0; l + 1 < L; ++l) {
        LevelGeom& v = g.lv[l];
        v.tk_pitch = round_up(v.w, 16);
        if (ORBGPU_PYR_STAGGER && l > 0 && (v.tk_pitch / 16) % 2 == 0) v.tk_pitch += 16;
        v.tk_ring = off;
        v.tk_ring_rows = C[l];
        off += l == 0 ? NC * g.tk_cstride0 : C[l] * v.tk_pitch;
    }
    g.lv[L - 1].tk_pitch = 0;
    g.lv[L - 1].tk_ring = 0;
    g.lv[L - 1].tk_ring_rows = 0;
    off += 16;
    if (off >= (1 << 20)) return fail(ORBGPU_ERR_UNSUPPORTED, "pyramid rings exceed the record offset range");
    const int sink = off;  // the last level's LDS stores land here (never read)
    off = round_up(off + 8 * (((g.lv[L - 1].w + 3) / 4 + 1) / 2), 16);
    g.tk_lds_tab = off;

    // --- plan table: row records of levels 1..L-1, then the ranges
    std::vector<int2>& tab = plan.tab;
    for (int l = 1; l < L; ++l) {
        LevelGeom& v = g.lv[l];
        v.tk_rec = (int)tab.size();
        for (int y = 0; y < v.h; ++y) {
            // slot offsets are multiples of 16: stored / 16 in 16 bits each
            const int a = slot_offset(g, l - 1, y0(l, y));
            const int b = slot_offset(g, l - 1, y1(l, y));
            tab.push_back(int2{(a >> 4) | ((b >> 4) << 16), ytab[(size_t)v.ytab_offset + y].y});
        }
    }
    // the kernel reads one record past a tick's last row (the second row of a
    // step at an odd end, discarded): it must hold a valid LDS offset
    for (int i = 0; i < 4; ++i) tab.push_back(int2{16 >> 4, 0});
    g.tk_rng = (int)tab.size() * 2;  // u32 index of the range table
    std::vector<uint32_t> rng;
    for (int k = 0; k < K; ++k) {
        for (int l = 1; l < L; ++l)
            for (const int n : {G[l], GT[l]}) {  // split the tick's rows into n contiguous runs
                const int a = p[k][l], b = p[k + 1][l], per = n ? (b - a + n - 1) / n : 0;
                for (int gi = 0; gi < n; ++gi) {
                    const int ra = std::min(a + gi * per, b), rb = std::min(ra + per, b);
                    const int d = l + 1 < L ? slot_offset(g, l, ra) : sink;
                    if (ra >= 2048 || rb - ra > 31 || (d >> 4) >= 65536)
                        return fail(ORBGPU_ERR_UNSUPPORTED, "pyramid range does not fit its packing");
                    rng.push_back((uint32_t)ra | (uint32_t)(rb - ra) << 11 | (uint32_t)(d >> 4) << 16);
                }
            }
        rng.push_back((uint32_t)(sink >> 4) << 16);  // the empty range of idle lanes
    }
    // ranges packed one per u32: row ra (11 bits) | row count (5) | LDS slot of row ra / 16 (16)
    if (rng.size() & 1) rng.push_back(0);
    for (size_t i = 0; i < rng.size(); i += 2) tab.push_back(int2{(int)rng[i], (int)rng[i + 1]});
    g.tk_tab_n = (int)tab.size();
    g.tk_lds_bytes = g.tk_lds_tab + 8 * g.tk_tab_n;
    if (g.tk_lds_bytes > 160 * 1024) return fail(ORBGPU_ERR_UNSUPPORTED, "pyramid plan exceeds 160 KiB of LDS");

    // --- column entries: (level, group, oct) in level order.  An oct is two
    // adjacent quads (8 pixels), always two real ones: a level with a
    // scalar-tail quad (the last quad, when w is not a multiple of 16) gets
    // the tail oct (Q-2, Q-1), whose quad B is the tail, and regular octs
    // (2o, 2o+1) over quads 0..Q-2; a level without one, over 0..Q-1.  An odd
    // count ends with the oct (last-1, last), which overlaps its neighbour
    // (both lanes write the same bytes).  The tail octs go last, from a wave
    // boundary, so the kernel's vertical-pass form is wave-uniform.
    struct Ent { int l, gi, qa, qb; };
    std::vector<Ent> ents, tails;
    for (int l = 1; l < L; ++l) {
        const int Q = (g.lv[l].w + 3) / 4;
        const bool has_tail = g.lv[l].qmain < Q;
        const int last = has_tail ? Q - 2 : Q - 1;  // last quad of the regular octs
        for (int gi = 0; gi < G[l]; ++gi) {
            for (int qa = 0; qa <= last; qa += 2) {
                const int a = std::min(qa, last - 1);
                ents.push_back(Ent{l, gi, a, a + 1});
            }
        }
        if (has_tail)
            for (int gi = 0; gi < GT[l]; ++gi) tails.push_back(Ent{l, -1 - gi, Q - 2, Q - 1});  // gi < 0: tail groups
    }
    if (tails.size() > 64) return fail(ORBGPU_ERR_UNSUPPORTED, "pyramid: more than 64 scalar-tail columns");
    while (!tails.empty() && ents.size() % 64 != 0) ents.push_back(Ent{0, 0, 0, 0});  // padding lanes
    ents.insert(ents.end(), tails.begin(), tails.end());
    const int n = (int)ents.size();
    const int cmax = 1024 - 64 * g.tk_pwaves;
    const int E = n <= cmax ? 1 : 2;
    const int CL = round_up((n + E - 1) / E, 64);
    if (E * CL < n || CL > cmax) return fail(ORBGPU_ERR_UNSUPPORTED, "pyramid levels too wide for one block");
    g.tk_e = E;
    g.tk_cwaves = CL / 64;
    g.tk_threads = 64 * (g.tk_cwaves + g.tk_pwaves);
    if (g.lv[0].tk_pitch != 16 * v4 || g.tk_cstride0 < T0 * g.lv[0].tk_pitch)
        return fail(ORBGPU_ERR_UNSUPPORTED, "level-0 ring layout");

    // per lane and entry: 9 int4 (pyramid.hip TickEnt)
    plan.ent.assign((size_t)CL * E * 9, int4{0, 0, 0, 0});
    for (int i = 0; i < CL * E; ++i) {
        int4* r = &plan.ent[(size_t)i * 9];
        if (i >= n) {
            r[0] = int4{slots, 0, 0, 0};  // empty range
            r[1] = int4{sink, -1, 0, 0};
            continue;
        }
        const Ent& en = ents[(size_t)i];
        if (en.l == 0) {  // padding before the tail wave
            r[0] = int4{slots, 0, 0, 0};
            r[1] = int4{sink, -1, 0, 0};
            continue;
        }
        const LevelGeom& v = g.lv[en.l];
        const bool last = en.l + 1 == L;
        const int qa = en.qa, qb = en.qb;
        if (qa < 0 || qb != qa + 1) return fail(ORBGPU_ERR_UNSUPPORTED, "pyramid: oct layout");
        const int tail = qb >= v.qmain ? 2 : 0;  // quad A is never a tail quad
        const int slot = en.gi >= 0 ? base_r[en.l] + en.gi : base_t[en.l] + (-1 - en.gi);
        r[0] = int4{slot, tail, v.tk_rec, last ? 0 : v.tk_pitch};
        r[1] = int4{last ? sink : v.tk_ring, last ? -1 : v.tk_ring + v.tk_ring_rows * v.tk_pitch, v.pitch,
                    (int)v.frame_bytes};
        const uint64_t o = (uint64_t)v.offset + 4u * (uint64_t)qa;
        if (o + (uint64_t)v.frame_bytes * (uint64_t)max_batch >= (1ull << 32))
            return fail(ORBGPU_ERR_UNSUPPORTED, "pyramid buffer beyond 4 GiB (32-bit store offsets)");
        r[2] = int4{(int)(uint32_t)o, 0, 4 * qa, en.l};
        const int4* ta = &ptab[(size_t)v.ptab_offset + 3 * (size_t)qa];
        const int4* tb = &ptab[(size_t)v.ptab_offset + 3 * (size_t)qb];
        for (int j = 0; j < 3; ++j) {
            r[3 + j] = ta[j];
            r[6 + j] = tb[j];
        }
    }
    return ORBGPU_OK;
}

// ---------------------------------------------------------------------------
// CPU emulation of pyramid_tick_kernel over a plan: the same LDS image, slots,
// records, ranges and per-lane entries, the same byte selection and
// fixed-point arithmetic.  Reads of a tick see the LDS as it was at the tick's
// start; every read checks that its slot still holds the expected row and no
// write of the same tick lands in a slot read during it, so a plan with a
// ring too small or a row scheduled too early fails here.
// ---------------------------------------------------------------------------
namespace {

inline uint32_t perm_b32(uint32_t s0, uint32_t s1, uint32_t sel) {  // v_perm_b32 (selectors 0..7, 12 = zero)
    const uint64_t v = ((uint64_t)s0 << 32) | s1;
    uint32_t out = 0;
    for (int i = 0; i < 4; ++i) {
        const uint32_t s = (sel >> (8 * i)) & 0xFF;
        const uint32_t b = s < 8 ? (uint32_t)(v >> (8 * s)) & 0xFF : 0u;
        out |= b << (8 * i);
    }
    return out;
}

inline uint32_t dot2_u16(uint32_t a, uint32_t b) {
    return (a & 0xFFFF) * (b & 0xFFFF) + (a >> 16) * (b >> 16);
}

}  // namespace

int emulate_pyramid(const Geom& g, const std::vector<int2>& ytab, const PyrPlan& plan, const uint8_t* img, size_t row0,
                    std::vector<std::vector<uint8_t>>& levels) {
    const int L = g.nlevels;
    levels.assign(L, {});
    for (int l = 1; l < L; ++l) levels[l].assign((size_t)g.lv[l].w * g.lv[l].h, 0);
    if (L < 2) return ORBGPU_OK;
    std::vector<uint8_t> lds((size_t)g.tk_lds_bytes, 0xA5);
    // owner of each 16-byte LDS row start: (level << 24) | row, -1 none
    std::vector<int> owner((size_t)g.tk_lds_bytes / 16 + 1, -1);
    std::memcpy(lds.data() + g.tk_lds_tab, plan.tab.data(), plan.tab.size() * sizeof(int2));
    const int2* tab = reinterpret_cast<const int2*>(lds.data() + g.tk_lds_tab);
    const LevelGeom& V0 = g.lv[0];
    const int T0 = g.tk_t0, H0 = V0.h;
    auto run_rows = [&](int c, std::vector<int>& offs) {  // the LDS rows a chunk's DMA writes
        for (int r = 0; r < T0; ++r) offs.push_back(slot_offset(g, 0, c * T0 + r));
    };
    auto stage = [&](int c) {  // chunk c lands (rows past the frame repeat its last row)
        const int cc = std::min(c, g.tk_k0 - 1);
        for (int r = 0; r < T0; ++r) {
            const int o = slot_offset(g, 0, c * T0 + r);
            std::memcpy(lds.data() + o, img + (size_t)std::min(cc * T0 + r, H0 - 1) * row0, (size_t)V0.w);
            owner[(size_t)o / 16] = c * T0 + r;
        }
    };
    stage(0);
    const int CL = g.tk_cwaves * 64, E = g.tk_e;
    struct W { int off; uint32_t v; int own; };
    for (int k = 0; k < g.tk_ticks; ++k) {
        std::vector<W> writes;
        std::vector<int> reads;  // LDS row offsets read in this tick
        for (int lane = 0; lane < CL; ++lane)
            for (int e = 0; e < E; ++e) {
                const int4* r = &plan.ent[((size_t)e * CL + lane) * 9];
                const uint32_t rg = reinterpret_cast<const uint32_t*>(tab)[g.tk_rng + k * g.tk_rs + r[0].x];
                const int ra = (int)(rg & 0x7FF), rb = ra + (int)((rg >> 11) & 31);
                if (ra >= rb) continue;
                const int l = r[2].w;
                const LevelGeom& v = g.lv[l];
                const int q0 = r[2].z / 4;  // quads q0, q0 + 1
                int d = (int)(rg >> 16) << 4;
                for (int y = ra; y < rb; ++y) {
                    const int2 rec = tab[r[0].z + y];
                    const int offs[2] = {(rec.x & 0xFFFF) << 4, (int)((uint32_t)rec.x >> 16) << 4};
                    const int2 yt = ytab[(size_t)v.ytab_offset + y];
                    const int srow[2] = {yt.x & 0xFFFF, yt.x >> 16};
                    for (int s = 0; s < 2; ++s) {
                        if (owner[(size_t)offs[s] / 16] != (((l - 1) << 24) | srow[s]))
                            return fail(ORBGPU_ERR_UNSUPPORTED, "pyramid plan: level " + std::to_string(l) + " row " +
                                                                    std::to_string(y) + " reads a slot not holding its source row");
                        reads.push_back(offs[s]);
                    }
                    uint32_t outq[2];
                    for (int qq = 0; qq < 2; ++qq) {
                    const int4* t = r + 3 + 3 * qq;
                    const int w0 = t[0].x;
                    const uint32_t wt[4] = {(uint32_t)t[0].y, (uint32_t)t[0].z, (uint32_t)t[0].w, (uint32_t)t[1].x};
                    const uint32_t sel[4] = {(uint32_t)t[1].y, (uint32_t)t[1].z, (uint32_t)t[1].w, (uint32_t)t[2].x};
                    uint32_t h[2][4];
                    for (int s = 0; s < 2; ++s) {
                        uint32_t dw[3];
                        std::memcpy(dw, lds.data() + offs[s] + w0, 12);
                        for (int j = 0; j < 4; ++j) {
                            const uint32_t pp = j < 3 ? perm_b32(dw[1], dw[0], sel[j]) : perm_b32(dw[2], dw[1], sel[j]);
                            h[s][j] = dot2_u16(pp, wt[j]);
                        }
                    }
                    const uint32_t bp = (uint32_t)rec.y, b0 = bp & 0xFFFF, b1 = bp >> 16;
                    uint32_t out = 0;
                    for (int j = 0; j < 4; ++j) {
                        uint32_t o;
                        if ((r[0].y >> qq) & 1)  // FixedPtCast<int, uchar, 22>
                            o = ((h[0][j] >> 12) * b0 + (h[1][j] >> 12) * b1 + (1u << 21)) >> 22;
                        else  // VResizeLinearVec_32s8u
                            o = ((((h[0][j] >> 16) * b0 + (2u << 16)) >> 16) + (((h[1][j] >> 16) * b1) >> 16)) >> 2;
                        out |= (o & 0xFF) << (8 * j);
                    }
                    outq[qq] = out;
                    const int q = q0 + qq;
                    for (int j = 0; j < 4 && 4 * q + j < v.w; ++j)
                        levels[l][(size_t)y * v.w + 4 * q + j] = (uint8_t)(out >> (8 * j));
                    }
                    if (l + 1 < L && d != slot_offset(g, l, y))
                        return fail(ORBGPU_ERR_UNSUPPORTED, "pyramid plan: destination is not the row's slot");
                    for (int qq = 0; qq < 2; ++qq)
                        writes.push_back(W{d + 4 * (q0 + qq), outq[qq], l + 1 < L ? ((l << 24) | y) : -1});
                    d += r[0].w;
                    if (d == r[1].y) d = r[1].x;
                }
            }
        // everything written during the tick -- the levels' new rows, chunk
        // k+1 landing and chunk k+2 in flight -- must miss the rows it reads
        std::sort(reads.begin(), reads.end());
        auto was_read = [&](int o) { return std::binary_search(reads.begin(), reads.end(), o); };
        std::vector<int> dma;
        run_rows(k + 1, dma);
        run_rows(k + 2, dma);
        for (int o : dma)
            if (was_read(o)) return fail(ORBGPU_ERR_UNSUPPORTED, "pyramid plan: a chunk lands in a slot in use");
        for (const W& w : writes) {
            if (w.own >= 0) {
                const int o = w.off & ~15;
                if (was_read(o)) return fail(ORBGPU_ERR_UNSUPPORTED, "pyramid plan: row overwrites a slot in use");
                owner[(size_t)o / 16] = w.own;
            }
            std::memcpy(lds.data() + w.off, &w.v, 4);
        }
        stage(k + 1);
    }
    return ORBGPU_OK;
}

}  // namespace orbgpu
