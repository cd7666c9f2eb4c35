/* orbx.h — C ABI of the MI355X-native ORB front-end (liborbx.so).
 *
 * Drop-in boundary for the hot path of the reference (zackLiuzz/MY_ORB_SLAM2).  Each entry
 * point names the reference interface it replaces (file:line relative to the reference
 * root).  Plain pointers and sizes only; no OpenCV, no torch types.  All functions return
 * an orbx_status (0 = ok, < 0 = error) and are safe to call from several host threads: a
 * handle serialises its own calls (an ORBextractor is not re-entrant in the reference either:
 * its pyramid is mutable state, include/ORBextractor.h:85), and a call waits only for its own
 * handle's work, never for the whole device (Tracking, LocalMapping and LoopClosing call the
 * hot path concurrently, src/System.cc:91-101).
 *
 * Numerics: bit-exact with the CPU restatement in oracle/ (same keypoints, angles,
 * descriptors, pyramid bytes, stereo outputs); see DESIGN.md for the OpenCV 3.2 conventions.
 */
#ifndef ORBX_H
#define ORBX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef enum {
    ORBX_OK = 0,
    ORBX_ERR_INVALID = -1,      /* bad argument (null pointer, size, level ...) */
    ORBX_ERR_DEVICE = -2,       /* HIP runtime error / no GPU */
    ORBX_ERR_CAPACITY = -3,     /* output buffer too small (n_out holds the needed size) */
    ORBX_ERR_UNSUPPORTED = -4,  /* configuration outside the kernels' design limits */
    ORBX_ERR_STATE = -5         /* call order (e.g. stereo before extraction) */
} orbx_status;

/* cv::KeyPoint field order and size (28 bytes), so a std::vector<cv::KeyPoint> buffer can
 * be filled directly. */
typedef struct {
    float x, y;       /* pt (level-0 pixel coordinates)          */
    float size;       /* (int)(31 * scale[octave])               */
    float angle;      /* degrees, fastAtan2 of the intensity centroid */
    float response;   /* FAST score                              */
    int32_t octave;   /* pyramid level                           */
    int32_t class_id; /* -1                                      */
} orbx_keypoint;

typedef struct {
    int nfeatures;       /* ORBextractor.nFeatures                  */
    float scale_factor;  /* ORBextractor.scaleFactor                */
    int nlevels;         /* ORBextractor.nLevels (<= 16)            */
    int ini_th_fast;     /* ORBextractor.iniThFAST                  */
    int min_th_fast;     /* ORBextractor.minThFAST                  */
    int cv_simd;         /* 1: OpenCV 3.2 x86-64 SSE2 rounding in resize/GaussianBlur
                            (default); 0: OpenCV scalar formulas      */
    int max_batch;       /* images per batched call (device workspace sizing), >= 1 */
    int device;          /* HIP device ordinal                       */
} orbx_extractor_params;

typedef struct orbx_extractor orbx_extractor;

/* Replaces ORB_SLAM2::ORBextractor::ORBextractor (src/ORBextractor.cc:410-470).
 * Device workspace is allocated lazily on the first call for a given image size. */
orbx_status orbx_extractor_create(const orbx_extractor_params* params, orbx_extractor** out);
orbx_status orbx_extractor_destroy(orbx_extractor* h);

/* ORBextractor getters (include/ORBextractor.h:63-83); arrays hold nlevels floats. */
orbx_status orbx_extractor_tables(const orbx_extractor* h, float* scale, float* inv_scale,
                                  float* sigma2, float* inv_sigma2, int* features_per_level);

/* Replaces ORBextractor::operator() (src/ORBextractor.cc:1065-1127) for one host image.
 * img: 8-bit gray, `stride` bytes per row.  Writes min(n, kp_cap) keypoints and rows of
 * 32-byte descriptors; *n_out = n.  An empty image (w or h == 0) returns ORBX_OK with
 * *n_out = -1 and leaves the outputs untouched, like the reference's silent return. */
orbx_status orbx_extract(orbx_extractor* h, const uint8_t* img, int width, int height,
                         size_t stride, orbx_keypoint* kps, int kp_cap, uint8_t* desc,
                         int* n_out);

/* orbx_extract without the copies out: *kps / *desc point at the handle's own (pinned host)
 * output block, *n_out keypoints and n x 32 descriptor bytes, valid until the next call that
 * uses this handle (an extraction, or orbx_stereo_match with it as either view).  The facade's
 * ORBextractor::operator() (integration/ORBextractor.h) copies them straight into its
 * std::vector<cv::KeyPoint> and descriptor cv::Mat.  Empty image: *n_out = -1, NULL views. */
orbx_status orbx_extract_view(orbx_extractor* h, const uint8_t* img, int width, int height,
                              size_t stride, const orbx_keypoint** kps, const uint8_t** desc,
                              int* n_out);

/* Build the geometry and device workspace for width x height images and up to `batch`
 * images per call (otherwise done lazily by the first call); *kp_cap = keypoint slots per
 * image in the batched outputs. */
orbx_status orbx_extractor_prepare(orbx_extractor* h, int width, int height, int batch,
                                   int* kp_cap);

/* mvImagePyramid[level] (include/ORBextractor.h:85) of image `index` of the last call,
 * copied to host (w*h bytes, tightly packed). */
orbx_status orbx_pyramid_level(orbx_extractor* h, int index, int level, uint8_t* out,
                               int* width, int* height);

/* ORBextractor::mvImagePyramid as the reference keeps it: filled by every operator()
 * (src/ORBextractor.cc:1129-1154, sized in the constructor at :433).  With host_pyramid on,
 * every orbx_extract / orbx_extract_view on the handle also copies its image's pyramid (all
 * levels, 1.51 MB at KITTI size) into a pinned host block of the handle's own, in the same
 * device sequence (the DMA runs beside the FAST / octree / descriptor kernels), and
 * orbx_host_pyramid_view then points at it: level l is height[l] rows of width[l] bytes,
 * step[l] bytes apart (the layout of a cv::Mat ROI, like the reference's levels, which are
 * views into a bordered image).  The block stays valid until the next orbx_extract(_view) on
 * the handle or its destruction; no other call writes it.  ORBX_ERR_STATE when the last such
 * call ran with host_pyramid off (the default) or failed.  The drop-in facade
 * (integration/ORBextractor.h) turns it on in its constructor. */
orbx_status orbx_extractor_host_pyramid(orbx_extractor* h, int on);
/* A counter that changes whenever the handle's pyramids do (every extraction or stereo frame on
 * it, a workspace regrowth): a caller that keeps (handle, image index) as the source of a view's
 * pyramid (the facade after ExtractStereo) detects that the source moved on. */
uint64_t orbx_extractor_serial(const orbx_extractor* h);
typedef struct {
    int nlevels;
    const uint8_t* data[16];
    int width[16], height[16];
    size_t step[16];
} orbx_host_pyramid;
orbx_status orbx_host_pyramid_view(const orbx_extractor* h, orbx_host_pyramid* out);

/* The 7x7 Gaussian of level `level` that the descriptors sample (the `workingMat` clone
 * blurred at src/ORBextractor.cc:1107-1108), copied to host like orbx_pyramid_level. */
orbx_status orbx_blur_level(orbx_extractor* h, int index, int level, uint8_t* out, int* width,
                            int* height);

/* ---- batched, device-resident API (throughput path) -------------------------------------
 * d_imgs: `batch` images in device memory, image i at d_imgs + i*batch_stride, rows
 * `stride` bytes apart.  Results stay in the handle's workspace; orbx_batch_view exposes
 * them as device pointers.  `stream` is the hipStream_t the call is ordered on (0 = the null
 * stream): its kernels run there, except the extraction's side branch, which is forked from
 * and joined back into it by events (orbx_extractor_set_overlap).  Calls that consume another
 * call's results (stereo after both extractions) must be on the same stream or ordered by
 * the caller. */
orbx_status orbx_extract_batch_device(orbx_extractor* h, const uint8_t* d_imgs, int batch,
                                      int width, int height, size_t stride,
                                      size_t batch_stride, void* stream);

/* ---- resident inputs: level 0 of the pyramid is the input buffer ----------------------
 * The extractor's pyramid level 0 (mvImagePyramid[0]) of image i lives at
 * *d_level0 + i * *image_stride, rows *pitch bytes apart (64-byte aligned, pitch >= width + 4).
 * A caller that writes its images there (an H2D copy straight from the camera buffer, or a
 * kernel) runs the extraction on them without the device-side copy of the input the other
 * batched entry points make: orbx_extract_batch_resident / orbx_stereo_frames_resident
 * (left views in images [0, B), right views in [B, 2B)).  Prepares the workspace for `batch`
 * images of width x height; the view stays valid until a call with another size or a larger
 * batch.  orbx_extract uses the same path for its host image. */
orbx_status orbx_batch_input_view(orbx_extractor* h, int width, int height, int batch,
                                  uint8_t** d_level0, size_t* pitch, size_t* image_stride);
orbx_status orbx_extract_batch_resident(orbx_extractor* h, int batch, void* stream);
orbx_status orbx_stereo_frames_resident(orbx_extractor* h, int batch, float mbf, float mb,
                                        float* d_uRight, float* d_depth, int32_t* d_nvalid,
                                        void* stream);

typedef struct {
    int batch;              /* images in the last call                        */
    int kp_cap;             /* keypoint slots per image                       */
    orbx_keypoint* kps;     /* device [batch][kp_cap]                         */
    uint8_t* desc;          /* device [batch][kp_cap][32]                     */
    int32_t* nkp;           /* device [batch]                                 */
    uint8_t* pyramid;       /* device [batch][pyr_bytes]                      */
    size_t pyr_bytes;       /* bytes per image pyramid block                  */
    int level_w[16], level_h[16], level_pitch[16];
    size_t level_off[16];   /* byte offset of each level inside the block      */
} orbx_batch_view;

orbx_status orbx_batch_view_get(const orbx_extractor* h, orbx_batch_view* view);

/* Copy outputs of images [first, first+count) of the last batched call to host (waits for
 * the device): nkp[count], kps[count][kp_cap], desc[count][kp_cap][32]; any may be NULL. */
orbx_status orbx_batch_fetch(orbx_extractor* h, int first, int count, int32_t* nkp,
                             orbx_keypoint* kps, uint8_t* desc);

/* Replaces Frame::ComputeStereoMatches (src/Frame.cc:496-686) for the last orbx_extract
 * calls on `left` and `right` (same image size, same params).  mb is the baseline term the
 * reference reads at Frame.cc:534 (normally mbf/fx).  uRight/depth: n_left floats
 * (-1 = no match).  *n_valid = accepted matches. */
orbx_status orbx_stereo_match(orbx_extractor* left, orbx_extractor* right, float mbf, float mb,
                              float* uRight, float* depth, int n_left, int* n_valid);

/* The stereo Frame constructor's extraction and matching (Frame.cc:66-120: ExtractORB of both
 * views, Frame.cc:89-92, then ComputeStereoMatches, Frame.cc:496-686) in one call on ONE
 * handle: both host images go into the handle's pinned staging and, by one 2-D DMA, into the
 * level-0 slots of a two-image batch (left = image 0, right = image 1); the two extractions run
 * as that batch and the stereo match is appended, and the whole device sequence is replayed from
 * one HIP graph with one host wait.  The results are the same as two orbx_extract calls on two
 * handles followed by orbx_stereo_match.  Outputs point into the handle's pinned block, valid
 * until the next call that uses the handle; n[v] < 0 never happens (an empty image returns
 * ORBX_ERR_INVALID).  mb as in orbx_stereo_match. */
typedef struct {
    const orbx_keypoint* kps[2];  /* [view] (0 = left, 1 = right): n[view] keypoints          */
    const uint8_t* desc[2];       /* [view]: n[view] x 32 bytes                                 */
    int32_t n[2];
    const float* u_right;         /* n[0] floats (-1 = no match)                                */
    const float* depth;           /* n[0] floats                                                */
    int32_t n_valid;
} orbx_stereo_frame_out;

orbx_status orbx_stereo_frame_view(orbx_extractor* h, const uint8_t* left, size_t stride_left,
                                   const uint8_t* right, size_t stride_right, int width,
                                   int height, float mbf, float mb, orbx_stereo_frame_out* out);

/* The pyramid after orbx_stereo_frame_view (ORBextractor::mvImagePyramid, ORBextractor.h:85,
 * filled by every operator() in the reference, ORBextractor.cc:1129-1154).  Calls on several
 * sessions' handles that meet are served as one batch on the device's frame server, so the
 * frame's pyramids may live in the server's workspace, not the caller's.  The contract is the
 * same either way:
 *   keep_pyramid off (the default): after orbx_stereo_frame_view, orbx_pyramid_level on the
 *     handle returns ORBX_ERR_STATE, whether the frame ran alone or in a batch;
 *   keep_pyramid on: orbx_pyramid_level(h, 0, l, ...) returns level l of the left view and
 *     (h, 1, l, ...) of the right view, whether the frame ran alone or in a batch (a served
 *     frame's two pyramid blocks are copied device to device into the handle: about 3 MB at
 *     KITTI size).
 * Any other extraction on the handle (orbx_extract, the batched calls) leaves the pyramids of
 * all its images, as before.  orbx_blurred_level needs the frame to have run on the handle
 * itself (it returns ORBX_ERR_STATE after a served frame). */
orbx_status orbx_extractor_keep_pyramid(orbx_extractor* h, int on);

/* Counters of the frame server that orbx_stereo_frame_view calls on handles with h's device and
 * parameters go to.  batches_of_size[m] = batches that held m frames (1 <= m <= 8);
 * batches_per_pair[i] = batches run in block pair i (the two pairs alternate);
 * peak_inflight = most batches (plus a lone call) on the device at once; users = live handles
 * that have called orbx_stereo_frame_view; resident = whether the server holds device / pinned
 * resources.  reset != 0 zeroes the counters after reading them. */
typedef struct {
    int64_t solo_calls;           /* calls that found the server idle and ran on their handle  */
    int64_t batches;
    int64_t served_frames;
    int64_t batches_of_size[9];
    int64_t batches_per_pair[2];
    int32_t peak_inflight;
    int32_t users;
    int32_t resident;
} orbx_frame_server_stats;
orbx_status orbx_frame_server_get_stats(const orbx_extractor* h, orbx_frame_server_stats* out,
                                        int reset);

/* Frees the frame server's resources (its two server handles with their workspaces, pinned
 * input / output blocks, device staging, graphs, stream) now; ORBX_ERR_STATE while a batch is
 * forming or running.  The next orbx_stereo_frame_view recreates them.  The server also
 * releases itself when the last handle that used it is destroyed. */
orbx_status orbx_frame_server_release(const orbx_extractor* h);

/* Batched stereo over the last orbx_extract_batch_device calls of both handles (pair i =
 * image i of each).  d_uRight/d_depth: device [batch][kp_cap] floats; d_nvalid: device
 * [batch] (may be NULL). */
orbx_status orbx_stereo_match_batch_device(orbx_extractor* left, orbx_extractor* right,
                                           float mbf, float mb, float* d_uRight,
                                           float* d_depth, int32_t* d_nvalid, void* stream);

/* The batched stereo Frame front-end (src/Frame.cc:72-102) on ONE handle: extracts the B
 * left and B right views as one batch of 2B images (images [0,B) left, [B,2B) right; both
 * views use the same ORBextractor parameters, as in the reference's Tracking.cc:136-139)
 * and runs ComputeStereoMatches on each pair.  Outputs: d_uRight/d_depth [batch][kp_cap],
 * d_nvalid [batch] (may be NULL); keypoints/descriptors via orbx_batch_view_get /
 * orbx_batch_fetch (left view = image i, right view = image B+i). */
orbx_status orbx_stereo_frames_device(orbx_extractor* h, const uint8_t* d_left,
                                      const uint8_t* d_right, int batch, int width, int height,
                                      size_t stride, size_t batch_stride, float mbf, float mb,
                                      float* d_uRight, float* d_depth, int32_t* d_nvalid,
                                      void* stream);

/* ---- descriptor matching (src/ORBmatcher.cc) ---------------------------------------------- */

/* ORBmatcher::DescriptorDistance (src/ORBmatcher.cc:1715-1731) on host memory. */
int orbx_descriptor_distance(const uint8_t* a, const uint8_t* b);

/* ---- overlap inside one extraction (no reference counterpart: scheduling only) ----------
 * The pyramid is a chain of launches (level l is resized from level l-1, ORBextractor.cc:
 * 1129-1154) whose small levels leave most of the device idle.  The first `levels` levels'
 * FAST (mode 1), + DistributeOctTree (2), + IC_Angle / rBRIEF (3), + level 0's blur (4,
 * images in place only) then run on the handle's second stream, forked by an event before
 * level `fork_level`'s launch and joined back before the other levels' orientation; mode 0
 * runs every kernel in sequence on the call's stream.
 * Outputs are identical in every mode.  mode < 0 restores the built-in default. */
orbx_status orbx_extractor_set_overlap(orbx_extractor* h, int mode, int fork_level, int levels);
orbx_status orbx_extractor_get_overlap(const orbx_extractor* h, int* mode, int* fork_level,
                                       int* levels);

/* ---- per-kernel timing (HIP events set by each kernel's own dispatch, hipExtLaunchKernel) - */
/* ORBX_K_LEVEL: every pyramid launch; ORBX_K_LEVEL0: the level-0 launch alone (a part of
 * ORBX_K_LEVEL, reported separately: it blurs the input, the others also resize). */
typedef enum {
    ORBX_K_LEVEL = 0, ORBX_K_FAST, ORBX_K_OCTREE, ORBX_K_ORIENT_DESC, ORBX_K_STEREO,
    ORBX_K_LEVEL0, ORBX_K_COUNT
} orbx_kernel_id;
orbx_status orbx_profile_enable(orbx_extractor* h, int on);
/* Waits for the recorded launches, returns per-kernel total ms and launch counts since the
 * last collect (arrays of ORBX_K_COUNT), and resets them.  Stereo launches are attributed
 * to the left handle. */
orbx_status orbx_profile_collect(orbx_extractor* h, double* total_ms, int64_t* launches);
const char* orbx_kernel_name(int id);

/* The launch geometry a batched call of `batch` images would use after
 * orbx_extractor_prepare (diagnostics; the parity tests pin the benchmarked geometry with
 * it): strip_rows[nlevels] = output rows per k_level strip walk of each level (0: the level
 * runs the tiled kernel), *stereo_split = workgroups per pair of a stereo launch over batch/2
 * pairs (orbx_stereo_frames_device). */
orbx_status orbx_extractor_launch_info(const orbx_extractor* h, int batch, int* strip_rows,
                                       int* stereo_split);

/* Library / device information.  orbx_version() ends in "orbx-src:<hash>", the hash of the
 * sources the library was built from (my_orb_slam2_amd/build.py). */
const char* orbx_version(void);
/* Text of the last failing HIP call on this thread ("" if none). */
const char* orbx_last_error(void);
orbx_status orbx_device_count(int* n);

#ifdef __cplusplus
}
#endif
#endif /* ORBX_H */
