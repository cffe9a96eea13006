/*
 * orbgpu.h -- C ABI of the MI355X-native ORB-SLAM2 front-end hot path.
 *
 * Drop-in boundary for the reference classes (paths relative to
 * /root/reference/ORB-SLAM2):
 *   ORBextractor            include/ORBextractor.h:47-111, src/ORBextractor.cpp
 *   ORBmatcher (subset)     include/ORBmatcher.h:37-141,  src/ORBmatcher.cpp
 * A header-only C++ adapter with the reference's class surface sits on top
 * of this ABI (include/orbslam2_amd/ORBextractor.h, ORBmatcher.h); the ctypes
 * / cgo-style binding a maintainer would add is shown in INTEGRATION.md.
 *
 * Conventions: every function returns an int status (ORBGPU_OK = 0, or a
 * negative ORBGPU_ERR_*); orbgpu_last_error() returns a thread-local message
 * for the last failure.  Plain pointers and sizes only.  "d_" pointers are
 * device (HBM) pointers; the rest are host pointers.  A handle may be used
 * by one thread at a time (like the reference's ORBextractor, which keeps
 * per-call state in mvImagePyramid).  Stream arguments are hipStream_t
 * passed as void* (NULL = the default stream).
 */
#ifndef ORBGPU_H
#define ORBGPU_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ABI version of this header.  Bumped whenever a struct the library writes
 * changes layout (round 5 appended orbgpu_extractor_info.device): a host
 * compares it with orbgpu_abi_version() of the library it loaded, or passes
 * its own struct size to orbgpu_extractor_get_info_sized. */
#define ORBGPU_ABI_VERSION 6

enum {
    ORBGPU_OK = 0,
    ORBGPU_ERR_ARG = -1,         /* invalid argument                         */
    ORBGPU_ERR_HIP = -2,         /* HIP runtime failure                      */
    ORBGPU_ERR_CAPACITY = -3,    /* an output / internal capacity exceeded   */
    ORBGPU_ERR_UNSUPPORTED = -4, /* geometry outside the supported envelope  */
    ORBGPU_ERR_NO_DEVICE = -5    /* no usable gfx950 device                  */
};

/* Bit-identical to cv::KeyPoint of OpenCV 2.4 (28 bytes):
 * Point2f pt; float size; float angle; float response; int octave; int class_id. */
typedef struct orbgpu_keypoint {
    float x, y, size, angle, response;
    int32_t octave, class_id;
} orbgpu_keypoint;

typedef struct orbgpu_extractor orbgpu_extractor;

typedef struct orbgpu_extractor_info {
    int nlevels;
    int width, height;              /* level-0 frame size                  */
    int max_batch;
    int max_keypoints;              /* per-frame upper bound of output N   */
    int level_width[32], level_height[32];
    int features_per_level[32];     /* mnFeaturesPerLevel                  */
    int level_capacity[32];         /* output slots per level: no frame yields more keypoints
                                       at that level (DistributeOctTree keeps at most
                                       mnFeaturesPerLevel + 3, or 4 per initial node)   */
    int device;                     /* HIP device ordinal the handle lives on           */
} orbgpu_extractor_info;

const char* orbgpu_last_error(void);
/* ORBGPU_ABI_VERSION of the header the library was built from. */
int orbgpu_abi_version(void);
/* 0 on success; fills the gfx arch name of the current device */
int orbgpu_device_arch(char* buf, int buflen);

/* ---------------------------------------------------------------------- */
/* ORBextractor                                                            */
/* ---------------------------------------------------------------------- */

/* Replaces ORBextractor::ORBextractor(nfeatures, scaleFactor, nlevels,
 * iniThFAST, minThFAST) (ORBextractor.h:51-52, ORBextractor.cpp:412-472).
 * width/height fix the frame geometry (the pyramid and cell grids are
 * precomputed); max_batch bounds orbgpu_extract_batch_device(). */
int orbgpu_extractor_create(int nfeatures, float scale_factor, int nlevels,
                            int ini_th_fast, int min_th_fast, int width, int height,
                            int max_batch, orbgpu_extractor** out);
/* The same on HIP device `device` (0 .. orbgpu_device_count()-1), whatever
 * the calling thread's current device: every later call on the handle runs on
 * that device (the reference runs one ORBextractor per camera thread,
 * src/Frame.cpp:84-87, src/Tracking.cpp:141-149; this places each on a GPU of
 * the host's choosing without the host linking HIP).  ORBGPU_ERR_ARG for an
 * ordinal outside the visible devices. */
int orbgpu_extractor_create_on_device(int device, int nfeatures, float scale_factor, int nlevels,
                                      int ini_th_fast, int min_th_fast, int width, int height,
                                      int max_batch, orbgpu_extractor** out);
int orbgpu_extractor_destroy(orbgpu_extractor* ex);

/* Device placement of the host-form calls (matchers, solvers, Initializer,
 * vocabulary; include/orbgpu_*.h): they run on the calling thread's device,
 * each (thread, device) with its own stream and staging.
 * orbgpu_set_thread_device makes `device` that device for the calling thread
 * (ORBGPU_ERR_ARG for an ordinal outside [0, count), ORBGPU_ERR_NO_DEVICE
 * without devices or for a non-gfx950 one); orbgpu_get_thread_device returns
 * it; orbgpu_device_count the visible devices (0 without any). */
int orbgpu_device_count(int* n);
int orbgpu_set_thread_device(int device);
int orbgpu_get_thread_device(int* device);
int orbgpu_extractor_get_info(const orbgpu_extractor* ex, orbgpu_extractor_info* info);
/* The same for a caller built against another header version: writes at most
 * info_size bytes (the caller's sizeof(orbgpu_extractor_info)), so an older,
 * shorter struct gets its own fields and nothing past them. */
int orbgpu_extractor_get_info_sized(const orbgpu_extractor* ex, orbgpu_extractor_info* info, size_t info_size);

/* GetScaleFactors / GetInverseScaleFactors / GetScaleSigmaSquares /
 * GetInverseScaleSigmaSquares (ORBextractor.h:63-83).  Arrays of nlevels. */
int orbgpu_extractor_get_scales(const orbgpu_extractor* ex, float* scale, float* inv_scale,
                                float* sigma2, float* inv_sigma2);

/* ORBextractor::operator()(image, mask, keypoints, descriptors)
 * (ORBextractor.h:56-61, ORBextractor.cpp:1053-1117), host to host, one frame.
 * image: CV_8UC1 width x height with row pitch `step` bytes.  Writes n <=
 * capacity keypoints and n x 32 descriptor bytes (levels 0..L-1 in order).
 * An empty image (NULL / zero size) returns ORBGPU_OK with *n = -1 and
 * touches no output, like the reference's early return (:1056). */
int orbgpu_extract(orbgpu_extractor* ex, const uint8_t* image, int width, int height, size_t step,
                   orbgpu_keypoint* keypoints, uint8_t* descriptors, int capacity, int* n);

/* The stereo Frame's two extractions (src/Frame.cpp:84-87: ExtractORB(0) and
 * ExtractORB(1) on two std::threads) from ONE calling thread: frame 0 is
 * issued on ex0's stream, then frame 1 on ex1's (its host staging overlaps
 * frame 0's kernels), then both are collected -- the two extractions overlap
 * on the GPU as with the two threads, without a thread spawn per frame (the
 * spawn + join alone, measured on the GPU box: median 30-53 us, slowest of
 * 1000 up to 660 us).  Outputs and errors as orbgpu_extract, per frame; both
 * images width x height; ex0 != ex1.  A NULL image gives that frame *n = -1. */
int orbgpu_extract_pair(orbgpu_extractor* ex0, const uint8_t* image0, size_t step0, orbgpu_keypoint* keypoints0,
                        uint8_t* descriptors0, int capacity0, int* n0, orbgpu_extractor* ex1, const uint8_t* image1,
                        size_t step1, orbgpu_keypoint* keypoints1, uint8_t* descriptors1, int capacity1, int* n1,
                        int width, int height);

/* Batched, HBM-resident form of operator(): frame b is at
 * d_images + b*frame_step with row pitch row_step.  Frame b's keypoints go
 * to d_kps + b*kp_capacity, descriptors to d_desc + b*kp_capacity*32, count
 * to d_counts[b].  kp_capacity must be >= info.max_keypoints.  Asynchronous
 * on `stream`; call orbgpu_extractor_sync() to collect internal errors. */
int orbgpu_extract_batch_device(orbgpu_extractor* ex, const uint8_t* d_images, int batch,
                                size_t row_step, size_t frame_step, orbgpu_keypoint* d_kps,
                                uint8_t* d_desc, int* d_counts, int kp_capacity, void* stream);

/* Synchronise `stream` and report any capacity overflow the kernels flagged
 * since the last call (ORBGPU_ERR_CAPACITY) -- never silently truncated. */
int orbgpu_extractor_sync(orbgpu_extractor* ex, void* stream);

/* Stage timing.  While enabled, every extraction records HIP events on its
 * own stream around the four launch groups [pyramid (levels 1..L-1), FAST
 * cells, octree, angle+blur+rBRIEF].  orbgpu_extractor_stage_times()
 * synchronises and returns the summed milliseconds per group over all
 * extractions since the last reset, and their count. */
int orbgpu_extractor_profile(orbgpu_extractor* ex, int enable);
int orbgpu_extractor_stage_times(orbgpu_extractor* ex, float* ms4, int* nbatches, int reset);

/* Pipelining hook (no reference equivalent): after every later batch
 * extraction the extractor records `event` (a hipEvent_t, or NULL to clear)
 * on its stream right after the launch group `stage` (0 pyramid, 1 FAST
 * cells, 2 octree, 3 describe), so a caller can start dependent or
 * independent work on another stream at that point, e.g. the previous
 * batch's matching once the pyramid pass (which wants the whole chip) is
 * done. */
int orbgpu_extractor_set_stage_event(orbgpu_extractor* ex, int stage, void* event);

/* Device-scope events for ordering streams of one GPU (the stage hook above,
 * a matcher stream behind the extraction stream): created with
 * hipEventDisableTiming | hipEventDisableSystemFence, so recording one does
 * not write the caches back to system scope -- a default event's marker
 * costs the stream about 7 us before its next kernel on the MI355X
 * (profiles/r06_notes_ab.txt r6x).  Kernel completion already makes a
 * kernel's writes visible to later kernels of the device; an event the host
 * synchronises on to read host memory must be a default one.  `stream` is a
 * hipStream_t (NULL: the calling thread's default stream). */
int orbgpu_device_event_create(void** event);
int orbgpu_device_event_destroy(void* event);
int orbgpu_device_event_record(void* event, void* stream);
int orbgpu_stream_wait_device_event(void* stream, void* event);

/* mvImagePyramid[level] of frame `frame` of the last extraction, copied to
 * host (ORBextractor.h:85; read by Frame::ComputeStereoMatches). */
int orbgpu_extractor_copy_level(orbgpu_extractor* ex, int frame, int level, uint8_t* dst,
                                size_t dst_step);
/* All levels of frame `frame` of the last extraction at once (the host
 * mvImagePyramid of ORBextractor): dst[l] / dst_step[l] for l < nlevels.
 * One pinned staging copy per level on the extractor's stream and one
 * synchronisation. */
int orbgpu_extractor_copy_levels(orbgpu_extractor* ex, int frame, uint8_t* const* dst, const size_t* dst_step);

/* ---------------------------------------------------------------------- */
/* ORBmatcher                                                              */
/* ---------------------------------------------------------------------- */

#define ORBGPU_MATCH_CHECK_ORI 1      /* mbCheckOrientation                 */
#define ORBGPU_MATCH_ANNOTATED_HISTO 2 /* 注释版 rotation-bin factor 1/30   */

/* ORBmatcher::DescriptorDistance (ORBmatcher.cpp:1838-1854) for n
 * descriptor pairs resident in HBM: d_dist[i] = popcount(a_i xor b_i). */
int orbgpu_hamming_pairs_device(const uint8_t* d_a, const uint8_t* d_b, int n, int* d_dist, void* stream);

/* Delivery of a batch's outputs to the host thread that consumes them (the
 * Tracking thread reads one Frame's mvKeys / mDescriptors,
 * src/Tracking.cpp:280-317): the B frames' rows -- `rows` holds B x cap rows
 * of row_bytes each (a multiple of 4), frame b's first counts[b] rows used --
 * packed back to back into `packed` (frame b at sum_{b' < b} counts[b']), so
 * a single copy of sum(counts) rows moves only used data.  Up to four
 * tensors per call (keypoints, descriptors, matches, ...), each with its own
 * counts (device pointers); asynchronous on `stream`. */
typedef struct orbgpu_pack_desc {
    const uint8_t* rows;
    uint8_t* packed;
    const int* counts;
    int row_bytes;
} orbgpu_pack_desc;
int orbgpu_pack_rows_device(int batch, int cap, int ntensors, const orbgpu_pack_desc* descs, void* stream);

/* Frame image bounds of the 64x48 feature grid: Frame::mnMinX, mnMaxX,
 * mnMinY, mnMaxY (Frame.cpp:505-530; [0,cols]x[0,rows] without distortion). */
typedef struct orbgpu_grid_bounds {
    float min_x, max_x, min_y, max_y;
} orbgpu_grid_bounds;

/* ORBmatcher(nnratio, checkOri).SearchForInitialization(F1, F2,
 * vbPrevMatched, vnMatches12, windowSize) (ORBmatcher.h:108,
 * ORBmatcher.cpp:474-590), batched over pairs; keypoints are F.mvKeysUn and
 * F2's grid is Frame::AssignFeaturesToGrid over `bounds` (Frame.cpp:241-259).
 * Pair b: F1 keypoints d_kps1 + b*stride1 (count d_n1[b], levels in
 * extractor order), descriptors d_desc1 + b*stride1*32; same for F2.
 * d_prev_xy (nullable): float2 per F1 keypoint at + b*stride1*2, read and
 * updated (vbPrevMatched); NULL means vbPrevMatched = F1 positions.
 * d_matches12: int per F1 keypoint at + b*stride1; d_nmatches[b].
 * Capacity: up to 2048 level-0 keypoints per frame (pairs above 512 run in
 * a second, larger-LDS pass, pairs above 1024 in a third one that reads F2's
 * descriptors from HBM; a pass is launched only when stride1 or stride2
 * exceeds the previous pass's limit).  A pair with more reports
 * d_nmatches[b] = -1 and all its matches12 = -1; the status is per pair,
 * nothing global. */
int orbgpu_search_for_initialization_batch_device(
    int batch, orbgpu_grid_bounds bounds,
    const orbgpu_keypoint* d_kps1, const uint8_t* d_desc1, const int* d_n1, size_t stride1,
    const orbgpu_keypoint* d_kps2, const uint8_t* d_desc2, const int* d_n2, size_t stride2,
    float* d_prev_xy, int window, float nnratio, int flags,
    int* d_matches12, int* d_nmatches, void* stream);

/* The same with max_level0 > 0: a bound the caller knows on every frame's
 * level-0 keypoints (e.g. orbgpu_extractor_info.level_capacity[0] of the
 * extractor that produced them), so the larger-LDS passes are launched only
 * when max_level0 exceeds 512 (1024); max_level0 = 0 is the form above.  A
 * pair above the last pass launched reports d_nmatches[b] = -1. */
int orbgpu_search_for_initialization_batch_device_bounded(
    int batch, orbgpu_grid_bounds bounds,
    const orbgpu_keypoint* d_kps1, const uint8_t* d_desc1, const int* d_n1, size_t stride1,
    const orbgpu_keypoint* d_kps2, const uint8_t* d_desc2, const int* d_n2, size_t stride2,
    float* d_prev_xy, int window, float nnratio, int flags, int max_level0,
    int* d_matches12, int* d_nmatches, void* stream);

/* The stream form, as Tracking runs the matcher on consecutive frames
 * (mInitialFrame, mCurrentFrame) = (F_{t-1}, F_t) (src/Tracking.cpp:768-769,
 * ORBmatcher.cpp:474-590): `batch` frames of one extraction at d_kps + b*stride
 * (descriptors d_desc + b*stride*32, counts d_n[b]); pair b matches F1 =
 * frame b-1 against F2 = frame b, and pair 0 matches the frame BEFORE the
 * batch -- d_prev_kps / d_prev_desc / *d_prev_n, read in place (e.g. the last
 * frame of the previous batch's output set, or a boundary frame received from
 * another GPU), so no copy of it into the batch is needed.  m12 row b
 * (d_matches12 + b*stride, F1's keypoints) and d_nmatches[b] as above;
 * d_prev_xy (nullable) is vbPrevMatched per pair at + b*stride*2.  The prev
 * frame's capacity must not exceed `stride`.  max_level0 as in _bounded, and
 * it must bound the prev frame's level-0 keypoints too (a boundary frame from
 * another extractor: pass the larger of the two extractors'
 * level_capacity[0]); a pair above it reports d_nmatches[b] = -1. */
int orbgpu_search_for_initialization_stream_device(
    int batch, orbgpu_grid_bounds bounds,
    const orbgpu_keypoint* d_kps, const uint8_t* d_desc, const int* d_n, size_t stride,
    const orbgpu_keypoint* d_prev_kps, const uint8_t* d_prev_desc, const int* d_prev_n,
    float* d_prev_xy, int window, float nnratio, int flags, int max_level0,
    int* d_matches12, int* d_nmatches, void* stream);

/* Host-pointer convenience form for one pair; returns nmatches in *n.
 * ORBGPU_ERR_CAPACITY (and *nmatches = 0) for more than 2048 level-0
 * keypoints in either frame. */
int orbgpu_search_for_initialization(orbgpu_grid_bounds bounds,
                                     const orbgpu_keypoint* kps1, const uint8_t* desc1, int n1,
                                     const orbgpu_keypoint* kps2, const uint8_t* desc2, int n2,
                                     float* prev_xy, int window, float nnratio, int flags,
                                     int* matches12, int* nmatches);

#ifdef __cplusplus
}
#endif
#endif
