/*
 * orbgpu_frame.h -- the Frame set-up steps between extraction and matching,
 * batched on the GPU (conventions as orbgpu.h):
 *   Frame::UndistortKeyPoints   src/Frame.cpp:462-496 (cv::undistortPoints)
 *   Frame::ComputeImageBounds   src/Frame.cpp:498-530 (host; once per camera)
 *   Frame::AssignFeaturesToGrid src/Frame.cpp:241-259, PosInGrid :434-444
 * The distortion follows OpenCV 2.4's cvUndistortPoints (5 fixed-point
 * iterations in double, P = K); parity against a real OpenCV build is
 * unpinned.
 */
#ifndef ORBGPU_FRAME_H
#define ORBGPU_FRAME_H

#include "orbgpu.h"

#ifdef __cplusplus
extern "C" {
#endif

#define ORBGPU_GRID_COLS 64 /* FRAME_GRID_COLS, include/Frame.h:36 */
#define ORBGPU_GRID_ROWS 48 /* FRAME_GRID_ROWS, include/Frame.h:37 */

/* mK (fx, fy, cx, cy) and mDistCoef (k1, k2, p1, p2[, k3]; ndist = 4 or 5). */
typedef struct orbgpu_camera {
    float fx, fy, cx, cy;
    float dist[5];
    int ndist;
} orbgpu_camera;

/* Frame::ComputeImageBounds: mnMinX, mnMaxX, mnMinY, mnMaxY. */
int orbgpu_compute_image_bounds(const orbgpu_camera* cam, int cols, int rows, orbgpu_grid_bounds* out);

/* Frame::UndistortKeyPoints for `batch` frames of one camera: frame b's
 * keypoints at d_kps + b*kp_capacity (d_counts[b] of them) -> mvKeysUn at
 * d_kps_un + b*kp_capacity (a copy when dist[0] == 0, as the reference). */
int orbgpu_undistort_keypoints_batch_device(const orbgpu_camera* cam, int batch, const orbgpu_keypoint* d_kps,
                                            const int* d_counts, int kp_capacity, orbgpu_keypoint* d_kps_un,
                                            void* stream);

/* Frame::AssignFeaturesToGrid: frame b's grid as CSR -- cell (i, j) =
 * i*ORBGPU_GRID_ROWS + j holds d_cell_items[b*kp_capacity + k] for k in
 * [d_cell_start[b*(C+1) + cell], d_cell_start[b*(C+1) + cell + 1]), C =
 * 64*48, keypoint indices in increasing order (mGrid[i][j]'s push order).
 * kp_capacity <= 4096. */
int orbgpu_assign_features_to_grid_batch_device(int batch, orbgpu_grid_bounds bounds, const orbgpu_keypoint* d_kps_un,
                                                const int* d_counts, int kp_capacity, int* d_cell_start,
                                                int* d_cell_items, void* stream);

#ifdef __cplusplus
}
#endif
#endif
