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
    uint8_t* dd = nullptr;
    int *dc = nullptr, *dw = nullptr, *dn = nullptr, *dfn = nullptr, *dfo = nullptr, *dff = nullptr, *dfc = nullptr,
        *dbw = nullptr, *dbc = nullptr;
    double *dwt = nullptr, *dbv = nullptr;
    auto cleanup = [&]() {
        void* ptrs[] = {dd, dc, dw, dn, dfn, dfo, dff, dfc, dbw, dbc, dwt, dbv};
        for (void* p : ptrs)
            if (p) (void)hipFree(p);
    };
    bool ok = hipMalloc((void**)&dd, 32 * (size_t)s) == hipSuccess && hipMalloc((void**)&dc, 4) == hipSuccess &&
              hipMalloc((void**)&dw, 4 * (size_t)s) == hipSuccess && hipMalloc((void**)&dn, 4 * (size_t)s) == hipSuccess &&
              hipMalloc((void**)&dfn, 4 * (size_t)s) == hipSuccess &&
              hipMalloc((void**)&dfo, 4 * (size_t)(s + 1)) == hipSuccess &&
              hipMalloc((void**)&dff, 4 * (size_t)s) == hipSuccess && hipMalloc((void**)&dfc, 4) == hipSuccess &&
              hipMalloc((void**)&dbw, 4 * (size_t)s) == hipSuccess && hipMalloc((void**)&dbc, 4) == hipSuccess &&
              hipMalloc((void**)&dwt, 8 * (size_t)s) == hipSuccess && hipMalloc((void**)&dbv, 8 * (size_t)s) == hipSuccess;
    if (!ok) {
        cleanup();
        return fail(ORBGPU_ERR_HIP, "device allocation failed");
    }
    ok = (n == 0 || hipMemcpy(dd, desc, 32 * (size_t)n, hipMemcpyHostToDevice) == hipSuccess) &&
         hipMemcpy(dc, &n, 4, hipMemcpyHostToDevice) == hipSuccess;
    if (ok) rc = orbgpu_bow_transform_batch_device(voc, 1, dd, dc, s, levelsup, dw, dn, dwt, dfn, dfo, dff, dfc, dbw,
                                                   dbv, dbc, nullptr);
    if (!ok || rc) {
        cleanup();
        return rc ? rc : fail(ORBGPU_ERR_HIP, "upload failed");
    }
    int nf = 0, nb = 0;
    ok = hipDeviceSynchronize() == hipSuccess && hipMemcpy(&nf, dfc, 4, hipMemcpyDeviceToHost) == hipSuccess &&
         hipMemcpy(&nb, dbc, 4, hipMemcpyDeviceToHost) == hipSuccess &&
         (n == 0 || (hipMemcpy(word, dw, 4 * (size_t)n, hipMemcpyDeviceToHost) == hipSuccess &&
                     hipMemcpy(node, dn, 4 * (size_t)n, hipMemcpyDeviceToHost) == hipSuccess &&
                     hipMemcpy(weight, dwt, 8 * (size_t)n, hipMemcpyDeviceToHost) == hipSuccess &&
                     hipMemcpy(fv_features, dff, 4 * (size_t)n, hipMemcpyDeviceToHost) == hipSuccess)) &&
         hipMemcpy(fv_nodes, dfn, 4 * (size_t)std::max(nf, 0), hipMemcpyDeviceToHost) == hipSuccess &&
         hipMemcpy(fv_offsets, dfo, 4 * (size_t)(nf + 1), hipMemcpyDeviceToHost) == hipSuccess &&
         hipMemcpy(bow_words, dbw, 4 * (size_t)std::max(nb, 0), hipMemcpyDeviceToHost) == hipSuccess &&
         hipMemcpy(bow_values, dbv, 8 * (size_t)std::max(nb, 0), hipMemcpyDeviceToHost) == hipSuccess;
    cleanup();
    if (!ok) return fail(ORBGPU_ERR_HIP, "transform failed");
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
    std::vector<void*> allocs;
    auto cleanup = [&]() {
        for (void* p : allocs) (void)hipFree(p);
    };
    auto up = [&](const void* src, size_t bytes) -> void* {
        void* d = nullptr;
        if (hipMalloc(&d, std::max<size_t>(bytes, 4)) != hipSuccess) return nullptr;
        allocs.push_back(d);
        if (src && bytes && hipMemcpy(d, src, bytes, hipMemcpyHostToDevice) != hipSuccess) return nullptr;
        return d;
    };
    orbgpu_bow_frame fr[2];
    const orbgpu_bow_frame* src[2] = {a, b};
    for (int i = 0; i < 2; ++i) {
        const orbgpu_bow_frame& s = *src[i];
        fr[i] = s;
        fr[i].fv_nodes = (const int*)up(s.fv_nodes, 4 * (size_t)s.fv_n);
        fr[i].fv_offsets = (const int*)up(s.fv_offsets, 4 * (size_t)(s.fv_n + 1));
        const int nfeat = s.fv_n ? s.fv_offsets[s.fv_n] : 0;
        fr[i].fv_features = (const int*)up(s.fv_features, 4 * (size_t)nfeat);
        fr[i].desc = (const uint8_t*)up(s.desc, 32 * (size_t)s.n);
        fr[i].angle = (const float*)up(s.angle, 4 * (size_t)s.n);
        fr[i].valid = (const uint8_t*)up(s.valid, (size_t)s.n);
        if (!fr[i].fv_nodes || !fr[i].fv_offsets || !fr[i].fv_features || !fr[i].desc || !fr[i].angle ||
            !fr[i].valid) {
            cleanup();
            return fail(ORBGPU_ERR_HIP, "upload failed");
        }
    }
    const int stride = std::max(std::max(a->n, b->n), 1);
    orbgpu_bow_frame* dA = (orbgpu_bow_frame*)up(&fr[0], sizeof(fr[0]));
    orbgpu_bow_frame* dB = (orbgpu_bow_frame*)up(&fr[1], sizeof(fr[1]));
    int* dm = (int*)up(nullptr, 4 * (size_t)stride);
    int* dn = (int*)up(nullptr, 4);
    if (!dA || !dB || !dm || !dn) {
        cleanup();
        return fail(ORBGPU_ERR_HIP, "allocation failed");
    }
    rc = orbgpu_search_by_bow_batch_device(mode, 1, dA, dB, nnratio, check_ori, stride, dm, dn, nullptr);
    const int nout = mode == ORBGPU_BOW_KF_F ? b->n : a->n;
    const bool ok = !rc && hipDeviceSynchronize() == hipSuccess &&
                    (nout == 0 || hipMemcpy(match, dm, 4 * (size_t)nout, hipMemcpyDeviceToHost) == hipSuccess) &&
                    hipMemcpy(nmatches, dn, 4, hipMemcpyDeviceToHost) == hipSuccess;
    cleanup();
    if (rc) return rc;
    if (!ok) return fail(ORBGPU_ERR_HIP, "SearchByBoW failed");
    return ORBGPU_OK;
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
    std::vector<void*> allocs;
    auto cleanup = [&]() {
        for (void* p : allocs) (void)hipFree(p);
    };
    bool ok = true;
    auto up = [&](const void* src_, size_t bytes) -> void* {
        void* d = nullptr;
        if (hipMalloc(&d, std::max<size_t>(bytes, 4)) != hipSuccess) {
            ok = false;
            return nullptr;
        }
        allocs.push_back(d);
        if (src_ && bytes && hipMemcpy(d, src_, bytes, hipMemcpyHostToDevice) != hipSuccess) ok = false;
        return d;
    };
    orbgpu_triangulation_pair d = P;
    orbgpu_bow_frame* dst[2] = {&d.kf1, &d.kf2};
    for (int i = 0; i < 2; ++i) {
        const orbgpu_bow_frame& s = *src[i];
        orbgpu_bow_frame& f = *dst[i];
        f.fv_nodes = (const int*)up(s.fv_nodes, 4 * (size_t)s.fv_n);
        f.fv_offsets = (const int*)up(s.fv_offsets, 4 * (size_t)(s.fv_n + 1));
        const int nfeat = s.fv_n ? s.fv_offsets[s.fv_n] : 0;
        f.fv_features = (const int*)up(s.fv_features, 4 * (size_t)nfeat);
        f.desc = (const uint8_t*)up(s.desc, 32 * (size_t)s.n);
        f.angle = (const float*)up(s.angle, 4 * (size_t)s.n);
        f.valid = (const uint8_t*)up(s.valid, (size_t)s.n);
    }
    d.kps1 = (const orbgpu_keypoint*)up(P.kps1, sizeof(orbgpu_keypoint) * (size_t)P.kf1.n);
    d.kps2 = (const orbgpu_keypoint*)up(P.kps2, sizeof(orbgpu_keypoint) * (size_t)P.kf2.n);
    d.u_right1 = P.u_right1 ? (const float*)up(P.u_right1, 4 * (size_t)P.kf1.n) : nullptr;
    d.u_right2 = P.u_right2 ? (const float*)up(P.u_right2, 4 * (size_t)P.kf2.n) : nullptr;
    const int stride = std::max(std::max(P.kf1.n, P.kf2.n), 1);
    orbgpu_triangulation_pair* dP = (orbgpu_triangulation_pair*)up(&d, sizeof(d));
    int* dm = (int*)up(nullptr, 4 * (size_t)stride);
    int* dn = (int*)up(nullptr, 4);
    if (!ok) {
        cleanup();
        return fail(ORBGPU_ERR_HIP, "upload failed");
    }
    rc = orbgpu_search_for_triangulation_batch_device(1, dP, check_ori, stride, dm, dn, nullptr);
    ok = !rc && hipDeviceSynchronize() == hipSuccess &&
         (P.kf1.n == 0 || hipMemcpy(match12, dm, 4 * (size_t)P.kf1.n, hipMemcpyDeviceToHost) == hipSuccess) &&
         hipMemcpy(nmatches, dn, 4, hipMemcpyDeviceToHost) == hipSuccess;
    cleanup();
    if (rc) return rc;
    if (!ok) return fail(ORBGPU_ERR_HIP, "SearchForTriangulation failed");
    return ORBGPU_OK;
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
    std::vector<void*> allocs;
    bool ok = true;
    auto up = [&](const void* src, size_t bytes) -> void* {
        void* d = nullptr;
        if (hipMalloc(&d, std::max<size_t>(bytes, 8)) != hipSuccess) {
            ok = false;
            return nullptr;
        }
        allocs.push_back(d);
        if (src && bytes && hipMemcpy(d, src, bytes, hipMemcpyHostToDevice) != hipSuccess) ok = false;
        return d;
    };
    const int* dqw = (const int*)up(q_words, 4 * (size_t)nq);
    const double* dqv = (const double*)up(q_values, 8 * (size_t)nq);
    const int* doff = (const int*)up(db_offsets, 4 * (size_t)(nkf + 1));
    const int* dw = (const int*)up(db_words, 4 * ndb);
    const double* dv = (const double*)up(db_values, 8 * ndb);
    int* dc = (int*)up(nullptr, 4 * (size_t)nkf);
    double* ds = (double*)up(nullptr, 8 * (size_t)nkf);
    auto cleanup = [&]() {
        for (void* p : allocs) (void)hipFree(p);
    };
    if (!ok) {
        cleanup();
        return fail(ORBGPU_ERR_HIP, "upload failed");
    }
    rc = orbgpu_bow_score_batch_device(scoring, dqw, dqv, nq, nkf, doff, dw, dv, dc, ds, nullptr);
    ok = !rc && hipDeviceSynchronize() == hipSuccess &&
         hipMemcpy(common, dc, 4 * (size_t)nkf, hipMemcpyDeviceToHost) == hipSuccess &&
         hipMemcpy(scores, ds, 8 * (size_t)nkf, hipMemcpyDeviceToHost) == hipSuccess;
    cleanup();
    if (rc) return rc;
    if (!ok) return fail(ORBGPU_ERR_HIP, "bow score failed");
    return ORBGPU_OK;
}

}  // extern "C"
