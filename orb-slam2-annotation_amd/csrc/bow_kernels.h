// bow_kernels.h -- device view of a DBoW2 vocabulary and the launchers of
// bow.hip.
#pragma once

#include <hip/hip_runtime.h>

#include "../../include/orbgpu_bow.h"

namespace orbgpu {

struct VocabDev {
    const uint8_t* desc;      // 32 bytes per node
    const int* child_start;   // children of node i: children[child_start[i] .. +child_count[i]) in file order
    const int* child_count;
    const int* children;
    const int* word_id;       // Node::word_id (0 unless declared a leaf)
    const double* weight;     // Node::weight
    int L, scoring, weighting;
};

int bow_max_stride();
hipError_t launch_bow_transform(const VocabDev& V, int batch, const uint8_t* desc, const int* counts, int stride,
                                int levelsup, int* word, int* node, double* weight, int* fv_nodes, int* fv_offsets,
                                int* fv_features, int* fv_n, int* bow_words, double* bow_values, int* bow_n,
                                hipStream_t stream);
hipError_t launch_search_by_bow(int mode, int batch, const orbgpu_bow_frame* a, const orbgpu_bow_frame* b,
                                float nnratio, int check_ori, int stride, int* match, int* nmatches,
                                hipStream_t stream);

hipError_t launch_bow_db_score(int scoring, const int* qw, const double* qv, int nq, int nkf, const int* off,
                               const int* dw, const double* dv, int* common, double* score, hipStream_t stream);
hipError_t launch_search_for_triangulation(int batch, const orbgpu_triangulation_pair* pairs, int check_ori, int stride,
                                          int* match, int* nmatches, hipStream_t stream);

}  // namespace orbgpu
