// bow.cpp -- host side of include/orbgpu_bow.h: the DBoW2 vocabulary (text
// loader with the reference's parsing semantics, HBM copy of the tree) and
// the transform / SearchByBoW drivers.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/orbgpu_bow.h"
#include "bow_kernels.h"
#include "host_common.h"
#include "host_ctx.h"

using namespace orbgpu;

struct orbgpu_vocabulary {
    orbgpu_vocabulary_info info{};
    // device copies
    uint8_t* d_desc = nullptr;
    int *d_child_start = nullptr, *d_child_count = nullptr, *d_children = nullptr, *d_word_id = nullptr;
    double* d_weight = nullptr;
    ~orbgpu_vocabulary() {
        void* ptrs[] = {d_desc, d_child_start, d_child_count, d_children, d_word_id, d_weight};
        for (void* p : ptrs)
            if (p) (void)hipFree(p);
    }
    VocabDev dev() const {
        return VocabDev{d_desc, d_child_start, d_child_count, d_children, d_word_id, d_weight, info.L, info.scoring,
                        info.weighting};
    }
};

namespace {

struct HostNode {
    int parent = 0;
    std::vector<int> children;
    uint8_t desc[32] = {};
    double weight = 0.0;  // DBoW2 Node(): weight(0), word_id(0)
    int word_id = 0;
};

int upload(orbgpu_vocabulary* v, const std::vector<HostNode>& nodes, int n_words) {
    const size_t n = nodes.size();
    std::vector<uint8_t> desc(32 * n);
    std::vector<int> cs(n), cc(n), ch, wid(n);
    std::vector<double> w(n);
    for (size_t i = 0; i < n; ++i) {
        std::memcpy(&desc[32 * i], nodes[i].desc, 32);
        cs[i] = (int)ch.size();
        cc[i] = (int)nodes[i].children.size();
        ch.insert(ch.end(), nodes[i].children.begin(), nodes[i].children.end());
        wid[i] = nodes[i].word_id;
        w[i] = nodes[i].weight;
    }
    if (ch.empty()) ch.push_back(0);
    ORB_HIP(hipMalloc((void**)&v->d_desc, desc.size()));
    ORB_HIP(hipMalloc((void**)&v->d_child_start, 4 * n));
    ORB_HIP(hipMalloc((void**)&v->d_child_count, 4 * n));
    ORB_HIP(hipMalloc((void**)&v->d_children, 4 * ch.size()));
    ORB_HIP(hipMalloc((void**)&v->d_word_id, 4 * n));
    ORB_HIP(hipMalloc((void**)&v->d_weight, 8 * n));
    ORB_HIP(hipMemcpy(v->d_desc, desc.data(), desc.size(), hipMemcpyHostToDevice));
    ORB_HIP(hipMemcpy(v->d_child_start, cs.data(), 4 * n, hipMemcpyHostToDevice));
    ORB_HIP(hipMemcpy(v->d_child_count, cc.data(), 4 * n, hipMemcpyHostToDevice));
    ORB_HIP(hipMemcpy(v->d_children, ch.data(), 4 * ch.size(), hipMemcpyHostToDevice));
    ORB_HIP(hipMemcpy(v->d_word_id, wid.data(), 4 * n, hipMemcpyHostToDevice));
    ORB_HIP(hipMemcpy(v->d_weight, w.data(), 8 * n, hipMemcpyHostToDevice));
    v->info.n_nodes = (int)n;
    v->info.n_words = n_words;
    return ORBGPU_OK;
}

int finish(std::vector<HostNode>& nodes, int k, int L, int scoring, int weighting, int n_words,
           orbgpu_vocabulary** out) {
    int rc = check_device();
    if (rc) return rc;
    orbgpu_vocabulary* v = new orbgpu_vocabulary();
    v->info.k = k;
    v->info.L = L;
    v->info.scoring = scoring;
    v->info.weighting = weighting;
    rc = upload(v, nodes, n_words);
    if (rc) {
        delete v;
        return rc;
    }
    *out = v;
    return ORBGPU_OK;
}

}  // namespace

extern "C" {

int orbgpu_vocabulary_load_text(const char* path, orbgpu_vocabulary** out) {
    if (!path || !out) return fail(ORBGPU_ERR_ARG, "NULL argument");
    *out = nullptr;
    // TemplatedVocabulary::loadFromTextFile (TemplatedVocabulary.h:1359-1448):
    // header "k L scoring weighting", then one node per line
    // "parent isLeaf d0 .. d31 weight"; nodes are numbered in file order.
    std::ifstream f(path);
    if (!f.is_open()) return fail(ORBGPU_ERR_ARG, std::string("cannot open ") + path);
    std::string line;
    std::getline(f, line);
    std::stringstream hs(line);
    int k = -1, L = -1, n1 = -1, n2 = -1;
    hs >> k >> L >> n1 >> n2;
    if (k < 0 || k > 20 || L < 1 || L > 10 || n1 < 0 || n1 > 5 || n2 < 0 || n2 > 3)
        return fail(ORBGPU_ERR_ARG, "vocabulary header out of range (not a DBoW2 text vocabulary)");
    std::vector<HostNode> nodes(1);
    int n_words = 0;
    while (!f.eof()) {  // the reference's loop: a trailing newline yields one empty node line
        std::getline(f, line);
        std::stringstream ls(line);
        const int nid = (int)nodes.size();
        nodes.emplace_back();
        int pid = 0, leaf = 0;
        ls >> pid;  // a failed extraction stores 0 (C++11)
        if (pid < 0 || pid >= nid) return fail(ORBGPU_ERR_ARG, "vocabulary node with an invalid parent");
        nodes[nid].parent = pid;
        nodes[pid].children.push_back(nid);
        ls >> leaf;
        for (int j = 0; j < 32; ++j) {
            int b = 0;
            if (ls >> b) nodes[nid].desc[j] = (uint8_t)b;
            else ls.clear();
        }
        double w = 0.0;
        ls >> w;
        nodes[nid].weight = w;
        if (leaf > 0) nodes[nid].word_id = n_words++;
    }
    return finish(nodes, k, L, n1, n2, n_words, out);
}

int orbgpu_vocabulary_load_binary(const char* path, orbgpu_vocabulary** out) {
    if (!path || !out) return fail(ORBGPU_ERR_ARG, "NULL argument");
    *out = nullptr;
    // TemplatedVocabulary::loadFromBinaryFile (TemplatedVocabulary.h:1477-1522):
    // header u32 nb_nodes (root included), u32 size_node, int k, int L, int
    // scoring, int weighting; then records of size_node bytes: int parent,
    // 32 descriptor bytes, float weight, bool isLeaf (saveToBinaryFile, :1527-1548).
    std::ifstream f(path, std::ios::in | std::ios::binary);
    if (!f.is_open()) return fail(ORBGPU_ERR_ARG, std::string("cannot open ") + path);
    uint32_t nb_nodes = 0, size_node = 0;
    int32_t hdr[4] = {0, 0, 0, 0};
    f.read(reinterpret_cast<char*>(&nb_nodes), 4);
    f.read(reinterpret_cast<char*>(&size_node), 4);
    f.read(reinterpret_cast<char*>(hdr), 16);
    if (!f) return fail(ORBGPU_ERR_ARG, "vocabulary file shorter than the binary header");
    const int k = hdr[0], L = hdr[1], scoring = hdr[2], weighting = hdr[3];
    if (k < 0 || k > 20 || L < 1 || L > 10 || scoring < 0 || scoring > 5 || weighting < 0 || weighting > 3)
        return fail(ORBGPU_ERR_ARG, "vocabulary header out of range (not a DBoW2 binary vocabulary)");
    if (size_node < 41) return fail(ORBGPU_ERR_ARG, "binary vocabulary record smaller than 41 bytes");
    if (nb_nodes > (1u << 26)) return fail(ORBGPU_ERR_ARG, "binary vocabulary node count out of range");
    // m_nodes.resize(nb_nodes + 1); nodes past the records stay default and unattached
    std::vector<HostNode> nodes((size_t)nb_nodes + 1);
    // The record buffer persists across iterations, as the reference's: its
    // `while (!f.eof())` loop runs once more after the last full record, on a
    // read of 0 bytes, and so processes that record a second time (a short
    // final read overwrites only its prefix).  A file with no record at all
    // processes the buffer as allocated -- uninitialised there, zeros here.
    std::vector<char> buf(size_node, 0);
    int n_words = 0;
    size_t nid = 1;
    while (!f.eof()) {
        f.read(buf.data(), size_node);
        if (nid >= nodes.size()) return fail(ORBGPU_ERR_ARG, "binary vocabulary holds more records than nb_nodes");
        int32_t pid;
        float w;
        std::memcpy(&pid, buf.data(), 4);
        std::memcpy(nodes[nid].desc, buf.data() + 4, 32);
        std::memcpy(&w, buf.data() + 36, 4);
        if (pid < 0 || (size_t)pid >= nid) return fail(ORBGPU_ERR_ARG, "vocabulary node with an invalid parent");
        nodes[nid].parent = pid;
        nodes[pid].children.push_back((int)nid);
        nodes[nid].weight = (double)w;
        if (buf[40]) nodes[nid].word_id = n_words++;
        ++nid;
    }
    return finish(nodes, k, L, scoring, weighting, n_words, out);
}

int orbgpu_vocabulary_create(int k, int L, int scoring, int weighting, int n, const int* parent, const int* is_leaf,
                             const uint8_t* desc, const double* weight, orbgpu_vocabulary** out) {
    if (!out || n < 0 || (n > 0 && (!parent || !is_leaf || !desc || !weight)))
        return fail(ORBGPU_ERR_ARG, "invalid argument");
    *out = nullptr;
    if (k < 0 || k > 20 || L < 1 || L > 10 || scoring < 0 || scoring > 5 || weighting < 0 || weighting > 3)
        return fail(ORBGPU_ERR_ARG, "vocabulary parameters out of range");
    std::vector<HostNode> nodes(1 + (size_t)n);
    int n_words = 0;
    for (int i = 0; i < n; ++i) {
        const int nid = i + 1;
        if (parent[i] < 0 || parent[i] >= nid) return fail(ORBGPU_ERR_ARG, "invalid parent (nodes in file order)");
        nodes[nid].parent = parent[i];
        nodes[parent[i]].children.push_back(nid);
        std::memcpy(nodes[nid].desc, desc + 32 * (size_t)i, 32);
        nodes[nid].weight = weight[i];
        if (is_leaf[i] > 0) nodes[nid].word_id = n_words++;
    }
    return finish(nodes, k, L, scoring, weighting, n_words, out);
}

int orbgpu_vocabulary_destroy(orbgpu_vocabulary* voc) {
    delete voc;
    return ORBGPU_OK;
}

int orbgpu_vocabulary_get_info(const orbgpu_vocabulary* voc, orbgpu_vocabulary_info* info) {
    if (!voc || !info) return fail(ORBGPU_ERR_ARG, "NULL argument");
    *info = voc->info;
    return ORBGPU_OK;
}

int orbgpu_bow_transform_batch_device(const orbgpu_vocabulary* voc, int batch, const uint8_t* d_desc,
                                      const int* d_counts, int stride, int levelsup, int* d_word, int* d_node,
                                      double* d_weight, int* d_fv_nodes, int* d_fv_offsets, int* d_fv_features,
                                      int* d_fv_n, int* d_bow_words, double* d_bow_values, int* d_bow_n,
                                      void* stream) {
    if (!voc || batch < 0 || stride <= 0 || stride > bow_max_stride() ||
        (batch > 0 && (!d_desc || !d_counts || !d_word || !d_node || !d_weight || !d_fv_nodes || !d_fv_offsets ||
                       !d_fv_features || !d_fv_n || !d_bow_words || !d_bow_values || !d_bow_n)))
        return fail(ORBGPU_ERR_ARG, "invalid argument (stride must be 1..4096)");
    int rc = check_device();
    if (rc) return rc;
    if (voc->info.n_words == 0) return fail(ORBGPU_ERR_ARG, "empty vocabulary");
    ORB_HIP(launch_bow_transform(voc->dev(), batch, d_desc, d_counts, stride, levelsup, d_word, d_node, d_weight,
                                 d_fv_nodes, d_fv_offsets, d_fv_features, d_fv_n, d_bow_words, d_bow_values, d_bow_n,
                                 (hipStream_t)stream));
    return ORBGPU_OK;
}

int orbgpu_bow_transform(const orbgpu_vocabulary* voc, int n, const uint8_t* desc, int levelsup, int* word, int* node,
                         double* weight, int* fv_nodes, int* fv_offsets, int* fv_features, int* fv_n,
                         int* bow_words, double* bow_values, int* bow_n) {
    if (!voc || n < 0 || n > bow_max_stride() || (n > 0 && !desc) || !word || !node || !weight || !fv_nodes ||
        !fv_offsets || !fv_features || !fv_n || !bow_words || !bow_values || !bow_n)
        return fail(ORBGPU_ERR_ARG, "invalid argument (n must be 0..4096)");
    int rc = check_device();
    if (rc) return rc;
    const int s = std::max(n, 1);
    HostCtx* ctx;
    if ((rc = host_ctx(&ctx))) return rc;
    HostCall call(*ctx);
    const uint8_t* dd;
    const int* dc;
    int *dw, *dn, *dfn, *dfo, *dff, *dfc, *dbw, *dbc;
    double *dwt, *dbv;
    rc = call.run([&](HostCall& A) {
        dd = A.inout(desc, 32 * (size_t)n, 32 * (size_t)s);
        dc = A.in(&n, 1);
        dfc = A.out<int>(1);
        dbc = A.out<int>(1);
        dw = A.out<int>(s);
        dn = A.out<int>(s);
        dwt = A.out<double>(s);
        dff = A.out<int>(s);
        dfn = A.out<int>(s);
        dfo = A.out<int>(s + 1);
        dbw = A.out<int>(s);
        dbv = A.out<double>(s);
    });
    if (rc) return rc;
    rc = orbgpu_bow_transform_batch_device(voc, 1, dd, dc, s, levelsup, dw, dn, dwt, dfn, dfo, dff, dfc, dbw, dbv,
                                           dbc, ctx->stream);
    if (rc) return rc;
    int nf = 0, nb = 0;
    std::vector<int> fvn(s), fvo(s + 1), bw(s);
    std::vector<double> bv(s);
    call.fetch(dfc, &nf, 4);
    call.fetch(dbc, &nb, 4);
    call.fetch(dw, word, 4 * (size_t)n);
    call.fetch(dn, node, 4 * (size_t)n);
    call.fetch(dwt, weight, 8 * (size_t)n);
    call.fetch(dff, fv_features, 4 * (size_t)n);
    call.fetch(dfn, fvn.data(), 4 * (size_t)s);
    call.fetch(dfo, fvo.data(), 4 * (size_t)(s + 1));
    call.fetch(dbw, bw.data(), 4 * (size_t)s);
    call.fetch(dbv, bv.data(), 8 * (size_t)s);
    if ((rc = call.finish())) return rc;
    nf = std::max(nf, 0);
    nb = std::max(nb, 0);
    std::memcpy(fv_nodes, fvn.data(), 4 * (size_t)nf);
    std::memcpy(fv_offsets, fvo.data(), 4 * (size_t)(nf + 1));
    std::memcpy(bow_words, bw.data(), 4 * (size_t)nb);
    std::memcpy(bow_values, bv.data(), 8 * (size_t)nb);
    *fv_n = nf;
    *bow_n = nb;
    return ORBGPU_OK;
}

int orbgpu_search_by_bow_batch_device(int mode, int batch, const orbgpu_bow_frame* d_a, const orbgpu_bow_frame* d_b,
                                      float nnratio, int check_ori, int stride, int* d_match, int* d_nmatches,
                                      void* stream) {
    if ((mode != ORBGPU_BOW_KF_F && mode != ORBGPU_BOW_KF_KF) || batch < 0 || stride <= 0 ||
        stride > bow_max_stride() || (batch > 0 && (!d_a || !d_b || !d_match || !d_nmatches)))
        return fail(ORBGPU_ERR_ARG, "invalid argument (stride must be 1..4096)");
    int rc = check_device();
    if (rc) return rc;
    ORB_HIP(launch_search_by_bow(mode, batch, d_a, d_b, nnratio, check_ori, stride, d_match, d_nmatches,
                                 (hipStream_t)stream));
    return ORBGPU_OK;
}

int orbgpu_search_by_bow(int mode, const orbgpu_bow_frame* a, const orbgpu_bow_frame* b, float nnratio, int check_ori,
                         int* match, int* nmatches) {
    if (!a || !b || !match || !nmatches) return fail(ORBGPU_ERR_ARG, "NULL argument");
    if (a->n < 0 || b->n < 0 || a->n > bow_max_stride() || b->n > bow_max_stride() || a->fv_n < 0 || b->fv_n < 0)
        return fail(ORBGPU_ERR_ARG, "frame sizes out of range (<= 4096 features)");
    int rc = check_device();
    if (rc) return rc;
    HostCtx* ctx;
    if ((rc = host_ctx(&ctx))) return rc;
    HostCall call(*ctx);
    const orbgpu_bow_frame* src[2] = {a, b};
    const int stride = std::max(std::max(a->n, b->n), 1);
    const orbgpu_bow_frame *dA, *dB;
    int *dm, *dn;
    rc = call.run([&](HostCall& A) {
        orbgpu_bow_frame fr[2];
        for (int i = 0; i < 2; ++i) {
            const orbgpu_bow_frame& s = *src[i];
            fr[i] = s;
            fr[i].fv_nodes = A.inout(s.fv_nodes, (size_t)s.fv_n);
            fr[i].fv_offsets = A.inout(s.fv_offsets, (size_t)(s.fv_n + 1));
            const int nfeat = s.fv_n ? s.fv_offsets[s.fv_n] : 0;
            fr[i].fv_features = A.inout(s.fv_features, (size_t)nfeat);
            fr[i].desc = A.inout(s.desc, 32 * (size_t)s.n);
            fr[i].angle = A.inout(s.angle, (size_t)s.n);
            fr[i].valid = A.inout(s.valid, (size_t)s.n);
        }
        dA = A.in(&fr[0], 1);
        dB = A.in(&fr[1], 1);
        dm = A.out<int>((size_t)stride);
        dn = A.out<int>(1);
    });
    if (rc) return rc;
    rc = orbgpu_search_by_bow_batch_device(mode, 1, dA, dB, nnratio, check_ori, stride, dm, dn, ctx->stream);
    if (rc) return rc;
    const int nout = mode == ORBGPU_BOW_KF_F ? b->n : a->n;
    call.fetch(dm, match, 4 * (size_t)nout);
    call.fetch(dn, nmatches, 4);
    return call.finish();
}

int orbgpu_search_for_triangulation_batch_device(int batch, const orbgpu_triangulation_pair* d_pairs, int check_ori,
                                                 int stride, int* d_match12, int* d_nmatches, void* stream) {
    if (batch < 0 || stride <= 0 || stride > bow_max_stride() ||
        (batch > 0 && (!d_pairs || !d_match12 || !d_nmatches)))
        return fail(ORBGPU_ERR_ARG, "invalid argument (stride must be 1..4096)");
    int rc = check_device();
    if (rc) return rc;
    ORB_HIP(launch_search_for_triangulation(batch, d_pairs, check_ori, stride, d_match12, d_nmatches,
                                            (hipStream_t)stream));
    return ORBGPU_OK;
}

int orbgpu_search_for_triangulation(const orbgpu_triangulation_pair* pair, int check_ori, int* match12,
                                    int* nmatches) {
    if (!pair || !match12 || !nmatches) return fail(ORBGPU_ERR_ARG, "NULL argument");
    const orbgpu_triangulation_pair& P = *pair;
    const orbgpu_bow_frame* src[2] = {&P.kf1, &P.kf2};
    for (const orbgpu_bow_frame* f : src) {
        if (f->n < 0 || f->n > bow_max_stride() || f->fv_n < 0)
            return fail(ORBGPU_ERR_ARG, "keyframe sizes out of range (<= 4096 features)");
        if (f->n > 0 && (!f->desc || !f->angle || !f->valid))
            return fail(ORBGPU_ERR_ARG, "missing descriptors / angles / valid flags");
        if (f->fv_n > 0 && (!f->fv_nodes || !f->fv_offsets || !f->fv_features))
            return fail(ORBGPU_ERR_ARG, "missing FeatureVector");
    }
    if ((P.kf1.n > 0 && !P.kps1) || (P.kf2.n > 0 && !P.kps2)) return fail(ORBGPU_ERR_ARG, "missing keypoints");
    int rc = check_device();
    if (rc) return rc;
    HostCtx* ctx;
    if ((rc = host_ctx(&ctx))) return rc;
    HostCall call(*ctx);
    const int stride = std::max(std::max(P.kf1.n, P.kf2.n), 1);
    const orbgpu_triangulation_pair* dP;
    int *dm, *dn;
    rc = call.run([&](HostCall& A) {
        orbgpu_triangulation_pair d = P;
        orbgpu_bow_frame* dst[2] = {&d.kf1, &d.kf2};
        for (int i = 0; i < 2; ++i) {
            const orbgpu_bow_frame& s = *src[i];
            orbgpu_bow_frame& f = *dst[i];
            f.fv_nodes = A.inout(s.fv_nodes, (size_t)s.fv_n);
            f.fv_offsets = A.inout(s.fv_offsets, (size_t)(s.fv_n + 1));
            const int nfeat = s.fv_n ? s.fv_offsets[s.fv_n] : 0;
            f.fv_features = A.inout(s.fv_features, (size_t)nfeat);
            f.desc = A.inout(s.desc, 32 * (size_t)s.n);
            f.angle = A.inout(s.angle, (size_t)s.n);
            f.valid = A.inout(s.valid, (size_t)s.n);
        }
        d.kps1 = A.inout(P.kps1, (size_t)P.kf1.n);
        d.kps2 = A.inout(P.kps2, (size_t)P.kf2.n);
        d.u_right1 = A.in(P.u_right1, (size_t)P.kf1.n);
        d.u_right2 = A.in(P.u_right2, (size_t)P.kf2.n);
        dP = A.in(&d, 1);
        dm = A.out<int>((size_t)stride);
        dn = A.out<int>(1);
    });
    if (rc) return rc;
    rc = orbgpu_search_for_triangulation_batch_device(1, dP, check_ori, stride, dm, dn, ctx->stream);
    if (rc) return rc;
    call.fetch(dm, match12, 4 * (size_t)P.kf1.n);
    call.fetch(dn, nmatches, 4);
    return call.finish();
}

int orbgpu_bow_score_batch_device(int scoring, const int* d_q_words, const double* d_q_values, int nq, int nkf,
                                  const int* d_db_offsets, const int* d_db_words, const double* d_db_values,
                                  int* d_common, double* d_scores, void* stream) {
    if (scoring < 0 || scoring > 5 || nq < 0 || nkf < 0 ||
        (nkf > 0 && (!d_db_offsets || !d_common || !d_scores)) || (nq > 0 && (!d_q_words || !d_q_values)))
        return fail(ORBGPU_ERR_ARG, "invalid argument");
    int rc = check_device();
    if (rc) return rc;
    ORB_HIP(launch_bow_db_score(scoring, d_q_words, d_q_values, nq, nkf, d_db_offsets, d_db_words, d_db_values,
                                d_common, d_scores, (hipStream_t)stream));
    return ORBGPU_OK;
}

int orbgpu_bow_score(int scoring, const int* q_words, const double* q_values, int nq, int nkf,
                     const int* db_offsets, const int* db_words, const double* db_values, int* common,
                     double* scores) {
    if (scoring < 0 || scoring > 5 || nq < 0 || nkf < 0 || (nkf > 0 && (!db_offsets || !common || !scores)) ||
        (nq > 0 && (!q_words || !q_values)))
        return fail(ORBGPU_ERR_ARG, "invalid argument");
    if (nkf == 0) return ORBGPU_OK;
    const size_t ndb = (size_t)db_offsets[nkf];
    if (ndb > 0 && (!db_words || !db_values)) return fail(ORBGPU_ERR_ARG, "missing keyframe words");
    int rc = check_device();
    if (rc) return rc;
    HostCtx* ctx;
    if ((rc = host_ctx(&ctx))) return rc;
    HostCall call(*ctx);
    const int *dqw, *doff, *dw;
    const double *dqv, *dv;
    int* dc;
    double* ds;
    rc = call.run([&](HostCall& A) {
        dqw = A.inout(q_words, (size_t)nq);
        dqv = A.inout(q_values, (size_t)nq);
        doff = A.in(db_offsets, (size_t)(nkf + 1));
        dw = A.inout(db_words, ndb);
        dv = A.inout(db_values, ndb);
        dc = A.out<int>((size_t)nkf);
        ds = A.out<double>((size_t)nkf);
    });
    if (rc) return rc;
    rc = orbgpu_bow_score_batch_device(scoring, dqw, dqv, nq, nkf, doff, dw, dv, dc, ds, ctx->stream);
    if (rc) return rc;
    call.fetch(dc, common, 4 * (size_t)nkf);
    call.fetch(ds, scores, 8 * (size_t)nkf);
    return call.finish();
}

}  // extern "C"
