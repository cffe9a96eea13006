// ransac_kernels.h -- launchers of the RANSAC kernels (sim3.hip).
#pragma once

#include <hip/hip_runtime.h>

#include "../../include/orbgpu_ransac.h"

namespace orbgpu {

size_t sim3_hyp_bytes();
// hyps: one slot per sample triplet (total_samples * sim3_hyp_bytes()); max_hyp >= every n_hyp
hipError_t launch_sim3_ransac(int batch, const orbgpu_sim3_problem* probs, int max_hyp, const float* X1,
                              const float* X2, const float* e1, const float* e2, const int* samples, void* hyps,
                              orbgpu_sim3_result* results, uint8_t* inliers, hipStream_t stream);

size_t pnp_hyp_bytes();
// hyps: one slot per sample 4-tuple; lists: one int per point (Refine() index lists)
hipError_t launch_pnp_ransac(int batch, const orbgpu_pnp_problem* probs, int max_hyp, const float* P3,
                             const float* P2, const float* maxerr, const int* samples, void* hyps, int* lists,
                             orbgpu_pnp_result* results, uint8_t* best_mask, uint8_t* refined_mask,
                             hipStream_t stream);

}  // namespace orbgpu
