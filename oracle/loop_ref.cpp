/*
 * loop_ref.cpp -- C++ restatement of LoopClosing::ComputeSim3's hot loop
 * for the loop-burst CPU baseline (TEST INFRASTRUCTURE ONLY: bench.py's
 * cpu_baseline leg and tests/ call it; the product never links it).
 *
 * It is the same algorithm as oracle/loop_ref.py + bow_ref.search_by_bow
 * (checked against them in tests/test_loop.py), in C++ so the CPU leg of
 * config 5 is timed on compiled code rather than on Python loops.
 *
 * Citations: T = /root/reference/ORB-SLAM2/Thirdparty/DBoW2/DBoW2/
 * TemplatedVocabulary.h, M = .../src/ORBmatcher.cpp, S3 = .../src/
 * Sim3Solver.cpp, LC = .../src/LoopClosing.cpp, R = .../Thirdparty/DBoW2/
 * DUtils/Random.cpp.
 *
 * * transform (T:1242-1283): descend from the root, at every level the
 *   first child (file order) with the smallest Hamming distance; the node
 *   passed at level L - levelsup is the FeatureVector node; features whose
 *   word weight is > 0 enter the FeatureVector (T:1151-1235).
 * * SearchByBoW(KF1, KF2) (M:604-743): merge walk over the common nodes in
 *   ascending order, TH_LOW strict, float ratio test, vbMatched2, rotation
 *   histogram (HISTO_LENGTH/360 factor, std::round) and ComputeThreeMaxima
 *   (M:1792-1833).
 * * Sim3Solver constructor (S3:37-107) and SetRansacParameters (S3:111-141),
 *   iterate (S3:147-221) through orbref_sim3_ransac (ransac_ref.cpp) one
 *   hypothesis at a time, with RandomInt (R:33-50) over glibc's TYPE_3
 *   generator held per query (random_r after srandom_r(seed): the same
 *   stream rand() gives after srand(seed)).
 * * ComputeSim3's round-robin (LC:339-356); the SearchBySim3/OptimizeSim3
 *   verification is taken to pass, as in the GPU burst.
 */
#include <cmath>
#include <cstdint>
#include <cstdlib>
#include <cstring>
#include <map>
#include <vector>

#include "orbref.h"

namespace {

int hamming32(const uint8_t* a, const uint8_t* b) {
    int d = 0;
    for (int i = 0; i < 4; ++i) {
        uint64_t x, y;
        std::memcpy(&x, a + 8 * i, 8);
        std::memcpy(&y, b + 8 * i, 8);
        d += __builtin_popcountll(x ^ y);
    }
    return d;
}

struct Voc {
    int k = 0, L = 0;
    std::vector<uint8_t> desc;        // 32 B per node, node 0 = root
    std::vector<double> weight;
    std::vector<int> word_id;
    std::vector<int> child_start, child_count, children;
};

using FeatVec = std::map<int, std::vector<int>>;

void transform(const Voc& v, const uint8_t* D, int n, int levelsup, int* words, int* nodes, double* weights,
               FeatVec* fv) {
    const int nid_level = v.L - levelsup;
    for (int i = 0; i < n; ++i) {
        int fin = 0, nid = 0, level = 0;
        while (v.child_count[fin] > 0) {
            ++level;
            const int cs = v.child_start[fin], cc = v.child_count[fin];
            int best = v.children[cs], bd = hamming32(D + 32 * i, &v.desc[32 * (size_t)best]);
            for (int c = 1; c < cc; ++c) {
                const int nd = v.children[cs + c];
                const int d = hamming32(D + 32 * i, &v.desc[32 * (size_t)nd]);
                if (d < bd) { bd = d; best = nd; }
            }
            fin = best;
            if (level == nid_level) nid = fin;
        }
        const double w = v.weight[fin];
        if (words) words[i] = v.word_id[fin];
        if (nodes) nodes[i] = nid;
        if (weights) weights[i] = w;
        if (fv && w > 0) (*fv)[nid].push_back(i);
    }
}

void three_maxima(const std::vector<std::vector<int>>& hist, int& i1, int& i2, int& i3) {
    int m1 = 0, m2 = 0, m3 = 0;
    i1 = i2 = i3 = -1;
    for (int i = 0; i < (int)hist.size(); ++i) {
        const int s = (int)hist[i].size();
        if (s > m1) { m3 = m2; m2 = m1; m1 = s; i3 = i2; i2 = i1; i1 = i; }
        else if (s > m2) { m3 = m2; m2 = s; i3 = i2; i2 = i; }
        else if (s > m3) { m3 = s; i3 = i; }
    }
    if (m2 < 0.1f * (float)m1) { i2 = -1; i3 = -1; }
    else if (m3 < 0.1f * (float)m1) { i3 = -1; }
}

// SearchByBoW(KF1, KF2) (M:604-743); match: int[n1]
int search_by_bow_kf_kf(const FeatVec& fv1, const uint8_t* d1, const float* a1, const uint8_t* v1, int n1,
                        const FeatVec& fv2, const uint8_t* d2, const float* a2, const uint8_t* v2, int n2,
                        float nnratio, bool check_ori, int* match) {
    const int HL = 30, TH_LOW = 50;
    const float factor = (float)HL / 360.0f;
    for (int i = 0; i < n1; ++i) match[i] = -1;
    std::vector<char> matched2(n2, 0);
    std::vector<std::vector<int>> hist(HL);
    int nm = 0;
    auto it1 = fv1.begin(), it2 = fv2.begin();
    while (it1 != fv1.end() && it2 != fv2.end()) {
        if (it1->first == it2->first) {
            for (int ia : it1->second) {
                if (!v1[ia]) continue;
                int b1 = 256, b2 = 256, bidx = -1;
                for (int ib : it2->second) {
                    if (matched2[ib] || !v2[ib]) continue;
                    const int d = hamming32(d1 + 32 * ia, d2 + 32 * ib);
                    if (d < b1) { b2 = b1; b1 = d; bidx = ib; }
                    else if (d < b2) b2 = d;
                }
                if (b1 < TH_LOW && (float)b1 < nnratio * (float)b2) {
                    match[ia] = bidx;
                    matched2[bidx] = 1;
                    if (check_ori) {
                        float rot = a1[ia] - a2[bidx];
                        if (rot < 0.0f) rot += 360.0f;
                        int bin = (int)std::round(rot * factor);
                        if (bin == HL) bin = 0;
                        hist[bin].push_back(ia);
                    }
                    ++nm;
                }
            }
            ++it1; ++it2;
        } else if (it1->first < it2->first) {
            it1 = fv1.lower_bound(it2->first);
        } else {
            it2 = fv2.lower_bound(it1->first);
        }
    }
    if (check_ori) {
        int i1, i2, i3;
        three_maxima(hist, i1, i2, i3);
        for (int i = 0; i < HL; ++i) {
            if (i == i1 || i == i2 || i == i3) continue;
            for (int idx : hist[i]) { match[idx] = -1; --nm; }
        }
    }
    return nm;
}

// SearchByBoW(KF, F) (M:205-348): the KeyFrame's features (side A, valid =
// it has a MapPoint that is not bad) against the Frame's (side B); a Frame
// keypoint already matched is skipped; match: int[nB] = the A feature
int search_by_bow_kf_f(const FeatVec& fva, const uint8_t* da, const float* aa, const uint8_t* va,
                       const FeatVec& fvb, const uint8_t* db, const float* ab, int nb, float nnratio,
                       bool check_ori, int* match) {
    const int HL = 30, TH_LOW = 50;
    const float factor = (float)HL / 360.0f;
    for (int i = 0; i < nb; ++i) match[i] = -1;
    std::vector<std::vector<int>> hist(HL);
    int nm = 0;
    auto ia_it = fva.begin(), ib_it = fvb.begin();
    while (ia_it != fva.end() && ib_it != fvb.end()) {
        if (ia_it->first == ib_it->first) {
            for (int ia : ia_it->second) {
                if (!va[ia]) continue;
                int b1 = 256, b2 = 256, bidx = -1;
                for (int ib : ib_it->second) {
                    if (match[ib] >= 0) continue;
                    const int d = hamming32(da + 32 * ia, db + 32 * ib);
                    if (d < b1) { b2 = b1; b1 = d; bidx = ib; }
                    else if (d < b2) b2 = d;
                }
                if (b1 <= TH_LOW && (float)b1 < nnratio * (float)b2) {
                    match[bidx] = ia;
                    if (check_ori) {
                        float rot = aa[ia] - ab[bidx];
                        if (rot < 0.0f) rot += 360.0f;
                        int bin = (int)std::round(rot * factor);
                        if (bin == HL) bin = 0;
                        hist[bin].push_back(bidx);
                    }
                    ++nm;
                }
            }
            ++ia_it; ++ib_it;
        } else if (ia_it->first < ib_it->first) {
            ia_it = fva.lower_bound(ib_it->first);
        } else {
            ib_it = fvb.lower_bound(ia_it->first);
        }
    }
    if (check_ori) {
        int i1, i2, i3;
        three_maxima(hist, i1, i2, i3);
        for (int i = 0; i < HL; ++i) {
            if (i == i1 || i == i2 || i == i3) continue;
            for (int idx : hist[i]) { match[idx] = -1; --nm; }
        }
    }
    return nm;
}

// float 3x3 * float 3-vector, double accumulation, rounded to float
void gemv_f32(const float* R, const float* X, float* out) {
    for (int r = 0; r < 3; ++r)
        out[r] = (float)(((double)R[3 * r] * (double)X[0] + (double)R[3 * r + 1] * (double)X[1]) +
                         (double)R[3 * r + 2] * (double)X[2]);
}

struct Solver {
    int N = 0, max_its = 0, iterations = 0, best = 0;
    std::vector<float> X1, X2, e1, e2;
    bool discarded = false;
};

int max_iterations(int N, int min_inliers, double probability, int max_its) {
    const float eps = (float)min_inliers / (float)N;
    int n_it;
    if (min_inliers == N) {
        n_it = 1;
    } else {
        const double v = std::log(1 - probability) / std::log(1 - std::pow((double)eps, 3));
        n_it = (std::isfinite(v) && std::fabs(v) < 2147483648.0) ? (int)std::ceil(v) : INT32_MIN;
    }
    return std::max(1, std::min(n_it, max_its));
}

struct Rng {
    struct random_data rd;
    char state[128];
    explicit Rng(unsigned seed) {
        std::memset(&rd, 0, sizeof(rd));
        initstate_r(seed, state, sizeof(state), &rd);
    }
    int random_int(int lo, int hi) {  // R:33-50
        int32_t r;
        random_r(&rd, &r);
        const int d = hi - lo + 1;
        return int(((double)r / ((double)RAND_MAX + 1.0)) * d) + lo;
    }
};

}  // namespace

struct orbref_vocabulary {
    Voc v;
};

extern "C" {

orbref_vocabulary* orbref_vocabulary_create(int k, int L, int n, const int32_t* parent, const int32_t* is_leaf,
                                            const uint8_t* desc, const double* weight) {
    auto* h = new orbref_vocabulary();
    Voc& v = h->v;
    v.k = k;
    v.L = L;
    const int nn = n + 1;
    v.desc.assign(32 * (size_t)nn, 0);
    std::memcpy(&v.desc[32], desc, 32 * (size_t)n);
    v.weight.assign(nn, 0.0);
    v.word_id.assign(nn, 0);
    v.child_count.assign(nn, 0);
    int words = 0;
    for (int i = 0; i < n; ++i) {
        v.weight[i + 1] = weight[i];
        if (is_leaf[i]) v.word_id[i + 1] = words++;
        v.child_count[parent[i]]++;
    }
    v.child_start.assign(nn, 0);
    for (int i = 1; i < nn; ++i) v.child_start[i] = v.child_start[i - 1] + v.child_count[i - 1];
    std::vector<int> fill(v.child_start);
    v.children.assign(n, 0);
    for (int i = 0; i < n; ++i) v.children[fill[parent[i]]++] = i + 1;  // file order within a parent
    return h;
}

void orbref_vocabulary_destroy(orbref_vocabulary* h) { delete h; }

void orbref_vocabulary_transform(const orbref_vocabulary* h, const uint8_t* desc, int n, int levelsup, int* words,
                                 int* nodes, double* weights) {
    transform(h->v, desc, n, levelsup, words, nodes, weights, nullptr);
}

int orbref_search_by_bow_kf_kf(const orbref_vocabulary* h, const uint8_t* d1, const float* a1, const uint8_t* v1,
                               int n1, const uint8_t* d2, const float* a2, const uint8_t* v2, int n2,
                               float nnratio, int check_ori, int* match) {
    FeatVec f1, f2;
    transform(h->v, d1, n1, 4, nullptr, nullptr, nullptr, &f1);
    transform(h->v, d2, n2, 4, nullptr, nullptr, nullptr, &f2);
    return search_by_bow_kf_kf(f1, d1, a1, v1, n1, f2, d2, a2, v2, n2, nnratio, check_ori != 0, match);
}

/* SearchByBoW(KF, F) on given FeatureVectors (Frame::ComputeBoW /
 * KeyFrame::ComputeBoW already run, as Tracking::TrackReferenceKeyFrame calls
 * it), each as a CSR: nodes[k] ascending, its features feats[start[k] ..
 * start[k+1]) in FeatureVector order. */
int orbref_search_by_bow_kf_f(const int* nodes_a, const int* start_a, const int* feats_a, int nn_a,
                              const uint8_t* da, const float* aa, const uint8_t* va, const int* nodes_b,
                              const int* start_b, const int* feats_b, int nn_b, const uint8_t* db, const float* ab,
                              int nb, float nnratio, int check_ori, int* match) {
    FeatVec fa, fb;
    for (int k = 0; k < nn_a; ++k) fa[nodes_a[k]].assign(feats_a + start_a[k], feats_a + start_a[k + 1]);
    for (int k = 0; k < nn_b; ++k) fb[nodes_b[k]].assign(feats_b + start_b[k], feats_b + start_b[k + 1]);
    return search_by_bow_kf_f(fa, da, aa, va, fb, db, ab, nb, nnratio, check_ori != 0, match);
}

/* One ComputeSim3 call (LC:273-356) for keyframe `cur` and candidates
 * cands[0..n_cand) of a scene laid out as synth.loop_burst_scene: desc
 * (n_kf, n_kp, 32), angle/valid (n_kf, n_kp), octave (n_kf, n_kp) i32,
 * mp_world (n_kf, n_kp, 3), Tcw (n_kf, 12), K (4), sigma2 (levels).
 * out: {matched, round, n_inliers, hypotheses}; nmatches: int[n_cand].
 * The _ex form also returns, when the pointers are not null: every
 * candidate's vpMatches12 (m12: int[n_cand][n_kp], -1 = none), the returned
 * Sim3 (pose: R12[9], t12[3], s12; zeros when no candidate returned one),
 * the solvers' (N, max_its, iterations, best inliers, discarded) per
 * candidate (cand_state: int[n_cand][5]) and the next random_r value of the
 * query's stream after its draws (rand_after). */
int orbref_compute_sim3_query(const orbref_vocabulary* h, int n_kp, const uint8_t* desc, const float* angle,
                              const int32_t* octave, const uint8_t* valid, const float* mp_world, const float* Tcw,
                              const float* K, const float* sigma2, int cur, const int* cands, int n_cand,
                              unsigned seed, int fix_scale, int* out, int* nmatches) {
    return orbref_compute_sim3_query_ex(h, n_kp, desc, angle, octave, valid, mp_world, Tcw, K, sigma2, cur, cands,
                                        n_cand, seed, fix_scale, out, nmatches, nullptr, nullptr, nullptr, nullptr);
}

int orbref_compute_sim3_query_ex(const orbref_vocabulary* h, int n_kp, const uint8_t* desc, const float* angle,
                                 const int32_t* octave, const uint8_t* valid, const float* mp_world,
                                 const float* Tcw, const float* K, const float* sigma2, int cur, const int* cands,
                                 int n_cand, unsigned seed, int fix_scale, int* out, int* nmatches, int* m12_out,
                                 float* pose, int* cand_state, int* rand_after) {
    const int min_matches = 20, min_inliers = 20, max_its = 300, per_call = 5;
    const double prob = 0.99;
    auto kf = [&](int i, size_t per) { return (size_t)i * (size_t)n_kp * per; };
    FeatVec fcur;
    transform(h->v, desc + kf(cur, 32), n_kp, 4, nullptr, nullptr, nullptr, &fcur);
    std::vector<Solver> sol(n_cand);
    std::vector<int> m12(n_kp);
    for (int c = 0; c < n_cand; ++c) {
        const int k2 = cands[c];
        FeatVec f2;
        transform(h->v, desc + kf(k2, 32), n_kp, 4, nullptr, nullptr, nullptr, &f2);
        const int nm = search_by_bow_kf_kf(fcur, desc + kf(cur, 32), angle + kf(cur, 1), valid + kf(cur, 1), n_kp,
                                           f2, desc + kf(k2, 32), angle + kf(k2, 1), valid + kf(k2, 1), n_kp, 0.75f,
                                           true, m12.data());
        nmatches[c] = nm;
        if (m12_out) std::memcpy(m12_out + (size_t)c * n_kp, m12.data(), sizeof(int) * (size_t)n_kp);
        Solver& s = sol[c];
        if (nm < min_matches) { s.discarded = true; continue; }
        // Sim3Solver ctor (S3:37-107)
        const float *R1 = Tcw + 12 * (size_t)cur, *t1 = R1 + 9, *R2 = Tcw + 12 * (size_t)k2, *t2 = R2 + 9;
        for (int i1 = 0; i1 < n_kp; ++i1) {
            const int i2 = m12[i1];
            if (i2 < 0 || !valid[kf(cur, 1) + i1] || !valid[kf(k2, 1) + i2]) continue;
            float a[3], b[3];
            gemv_f32(R1, mp_world + kf(cur, 3) + 3 * i1, a);
            gemv_f32(R2, mp_world + kf(k2, 3) + 3 * i2, b);
            for (int r = 0; r < 3; ++r) { s.X1.push_back(a[r] + t1[r]); s.X2.push_back(b[r] + t2[r]); }
            s.e1.push_back((float)(size_t)(9.210 * (double)sigma2[octave[kf(cur, 1) + i1]]));
            s.e2.push_back((float)(size_t)(9.210 * (double)sigma2[octave[kf(k2, 1) + i2]]));
        }
        s.N = (int)s.e1.size();
        s.max_its = s.N > 0 ? max_iterations(s.N, min_inliers, prob, max_its) : 0;
    }
    Rng rng(seed);
    int n_live = 0;
    for (auto& s : sol) n_live += !s.discarded;
    int rnd = -1;
    out[0] = -1; out[1] = -1; out[2] = 0;
    if (pose) std::memset(pose, 0, 13 * sizeof(float));
    int ints[4];
    float T[16], R[9], t[3], sc;
    std::vector<uint8_t> inl;
    bool matched = false;
    while (n_live > 0 && !matched) {
        ++rnd;
        for (int c = 0; c < n_cand && !matched; ++c) {
            Solver& s = sol[c];
            if (s.discarded) continue;
            bool found = false, no_more = false;
            if (s.N < min_inliers) {
                no_more = true;
            } else {
                inl.assign(s.N, 0);
                std::vector<int> avail(s.N);
                int cur_its = 0;
                while (s.iterations < s.max_its && cur_its < per_call) {
                    ++cur_its;
                    ++s.iterations;
                    for (int i = 0; i < s.N; ++i) avail[i] = i;
                    int na = s.N, smp[3];
                    for (int k = 0; k < 3; ++k) {
                        const int r = rng.random_int(0, na - 1);
                        smp[k] = avail[r];
                        avail[r] = avail[na - 1];
                        --na;
                    }
                    orbref_sim3_ransac(s.N, s.X1.data(), s.X2.data(), s.e1.data(), s.e2.data(), K, K, fix_scale,
                                       min_inliers, s.best, 1, smp, ints, T, R, t, &sc, inl.data());
                    if (ints[3] >= 0) s.best = ints[2];
                    if (ints[0]) { found = true; break; }
                }
                if (!found && s.iterations >= s.max_its) no_more = true;
            }
            if (no_more) { s.discarded = true; --n_live; }
            if (found) {
                out[0] = c; out[1] = rnd; out[2] = s.best;
                matched = true;
                if (pose) {
                    std::memcpy(pose, R, 9 * sizeof(float));
                    std::memcpy(pose + 9, t, 3 * sizeof(float));
                    pose[12] = sc;
                }
            }
        }
    }
    int hyp = 0;
    for (auto& s : sol) hyp += s.iterations;
    out[3] = hyp;
    if (cand_state)
        for (int c = 0; c < n_cand; ++c) {
            const Solver& s = sol[c];
            int* o = cand_state + 5 * c;
            o[0] = s.N; o[1] = s.max_its; o[2] = s.iterations; o[3] = s.best; o[4] = s.discarded ? 1 : 0;
        }
    if (rand_after) {
        int32_t r;
        random_r(&rng.rd, &r);
        *rand_after = r;
    }
    return out[0];
}

}  // extern "C"
