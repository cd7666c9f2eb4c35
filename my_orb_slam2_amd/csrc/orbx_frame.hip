// orbx_frame.hip — per-frame geometry around the matchers (include/orbx_frame.h).
//
//   k_undistort    one lane per keypoint: cvUndistortPoints (OpenCV 3.2) in double, the
//                  same __host__ __device__ routine the host uses for ComputeImageBounds
//   k_grid         Frame::AssignFeaturesToGrid as a counting sort, one workgroup per frame:
//                  cell of every keypoint (PosInGrid, std::round half away from zero in
//                  float), per-cell LDS counts, a block scan over the 3072 cells, an atomic
//                  fill, then each cell sorted by feature index (the push_back order)
#include <hip/hip_runtime.h>

#include <cmath>
#include <mutex>
#include <vector>

#include "../../include/orbx_frame.h"
#include "orbx_device.h"
#include "orbx_host.h"

using namespace orbx;

namespace {

struct UndistParams {
    double k[8];
    double fx, fy, cx, cy, ifx, ify;
    int iters;
};

__host__ __device__ inline void undistort_pt(const UndistParams& P, float xs, float ys,
                                             float& xo, float& yo) {
    const double* k = P.k;
    double x = xs, y = ys;
    const double x0 = x = (x - P.cx) * P.ifx;
    const double y0 = y = (y - P.cy) * P.ify;
    for (int j = 0; j < P.iters; j++) {   // compensate distortion iteratively
        const double r2 = x * x + y * y;
        const double icdist = (1 + ((k[7] * r2 + k[6]) * r2 + k[5]) * r2) /
                              (1 + ((k[4] * r2 + k[1]) * r2 + k[0]) * r2);
        const double deltaX = 2 * k[2] * x * y + k[3] * (r2 + 2 * x * x);
        const double deltaY = k[2] * (r2 + 2 * y * y) + 2 * k[3] * x * y;
        x = (x0 - deltaX) * icdist;
        y = (y0 - deltaY) * icdist;
    }
    // RR = P * I = K: xx = RR00*x + RR01*y + RR02, ..., ww = 1/(0*x + 0*y + 1)
    const double xx = P.fx * x + 0.0 * y + P.cx;
    const double yy = 0.0 * x + P.fy * y + P.cy;
    const double ww = 1. / (0.0 * x + 0.0 * y + 1.0);
    xo = (float)(xx * ww);
    yo = (float)(yy * ww);
}

bool make_params(const float* K4, const float* dist, int ndist, UndistParams& P) {
    if (!K4 || !dist || (ndist != 4 && ndist != 5 && ndist != 8)) return false;
    for (int i = 0; i < 8; ++i) P.k[i] = i < ndist ? (double)dist[i] : 0.0;
    P.fx = K4[0];
    P.fy = K4[1];
    P.cx = K4[2];
    P.cy = K4[3];
    P.ifx = 1. / P.fx;
    P.ify = 1. / P.fy;
    P.iters = 5;   // distortion coefficients given (cvUndistortPoints)
    return true;
}

__global__ __launch_bounds__(256) void k_undistort(UndistParams P, const orbx_keypoint* in,
                                                   int n, orbx_keypoint* out, int copy) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    orbx_keypoint kp = in[i];
    if (!copy) undistort_pt(P, kp.x, kp.y, kp.x, kp.y);
    out[i] = kp;
}

// PosInGrid (Frame.cc:407-417): round((x - mnMinX) * inv) in float, half away from zero.
__device__ inline int grid_cell(const orbx_keypoint& kp, int cols, int rows, float min_x,
                                float min_y, float inv_w, float inv_h) {
    const int px = (int)roundf((kp.x - min_x) * inv_w);
    const int py = (int)roundf((kp.y - min_y) * inv_h);
    if (px < 0 || px >= cols || py < 0 || py >= rows) return -1;
    return px * rows + py;
}

// One workgroup per frame: frame f's keypoints at kps + f*kp_stride (n_f = d_n[f] when given,
// else n), grid_off block at f*(cells+1), grid_feat at f*kp_stride.
__global__ __launch_bounds__(1024) void k_grid(const orbx_keypoint* __restrict__ kps, int n,
                                               const int32_t* __restrict__ d_n, int kp_stride,
                                               int cols, int rows, float min_x, float min_y,
                                               float inv_w, float inv_h,
                                               int32_t* __restrict__ grid_off,
                                               int32_t* __restrict__ grid_feat) {
    extern __shared__ int cnt[];   // cells + 1024 (scan partials)
    const int ncell = cols * rows, tid = threadIdx.x, f = blockIdx.x;
    if (d_n) n = min(max(d_n[f], 0), kp_stride);
    kps += (size_t)f * kp_stride;
    int32_t* off = grid_off + (size_t)f * (ncell + 1);
    int32_t* feat = grid_feat + (size_t)f * kp_stride;
    int* part = cnt + ncell;
    for (int c = tid; c < ncell; c += 1024) cnt[c] = 0;
    __syncthreads();
    for (int i = tid; i < n; i += 1024) {
        const int c = grid_cell(kps[i], cols, rows, min_x, min_y, inv_w, inv_h);
        if (c >= 0) atomicAdd(&cnt[c], 1);
    }
    __syncthreads();
    // exclusive scan: each thread sums a run of `per` cells, Hillis-Steele over the partials
    const int per = (ncell + 1023) / 1024, c0 = min(tid * per, ncell), c1 = min(c0 + per, ncell);
    int sum = 0;
    for (int c = c0; c < c1; ++c) sum += cnt[c];
    part[tid] = sum;
    __syncthreads();
    for (int d = 1; d < 1024; d <<= 1) {
        const int v = tid >= d ? part[tid - d] : 0;
        __syncthreads();
        part[tid] += v;
        __syncthreads();
    }
    int run = part[tid] - sum;
    for (int c = c0; c < c1; ++c) {
        const int v = cnt[c];
        cnt[c] = run;   // becomes the fill cursor
        off[c] = run;
        run += v;
    }
    if (tid == 1023) off[ncell] = part[1023];
    __syncthreads();
    for (int i = tid; i < n; i += 1024) {
        const int c = grid_cell(kps[i], cols, rows, min_x, min_y, inv_w, inv_h);
        if (c >= 0) feat[atomicAdd(&cnt[c], 1)] = i;
    }
    __syncthreads();
    // each cell ascending by feature index (the push_back order of Frame.cc:252-256)
    for (int c = tid; c < ncell; c += 1024) {
        const int b = off[c], e = cnt[c];
        for (int k = b + 1; k < e; ++k) {
            const int v = feat[k];
            int j = k - 1;
            while (j >= b && feat[j] > v) {
                feat[j + 1] = feat[j];
                --j;
            }
            feat[j + 1] = v;
        }
    }
}

__global__ __launch_bounds__(256) void k_undistort_batch(UndistParams P,
                                                         const orbx_keypoint* in, int kp_stride,
                                                         const int32_t* d_n,
                                                         orbx_keypoint* out, int copy) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x, f = blockIdx.y;
    if (i >= min(d_n[f], kp_stride)) return;
    const size_t k = (size_t)f * kp_stride + i;
    orbx_keypoint kp = in[k];
    if (!copy) undistort_pt(P, kp.x, kp.y, kp.x, kp.y);
    out[k] = kp;
}

// cvtColor(*2GRAY), OpenCV 3.2 RGB2Gray<uchar>: the three table terms summed with the
// 1 << 13 rounding constant, >> 14.  One thread per 4 output pixels.
__global__ __launch_bounds__(256) void k_gray(const uint8_t* __restrict__ src, int w, int h,
                                              size_t sstride, int scn, int rgb,
                                              uint8_t* __restrict__ dst, size_t dstride) {
    const int y = blockIdx.y;
    const int x0 = (blockIdx.x * 256 + threadIdx.x) * 4;
    if (x0 >= w) return;
    const uint8_t* s = src + (size_t)y * sstride + (size_t)x0 * scn;
    const int c0 = rgb ? 4899 : 1868, c2 = rgb ? 1868 : 4899;   // coeff of src[0], src[2]
    uint32_t out = 0;
    const int nx = min(4, w - x0);
#pragma unroll
    for (int j = 0; j < 4; ++j) {
        if (j < nx) {
            const int v = (c0 * s[j * scn] + 9617 * s[j * scn + 1] + c2 * s[j * scn + 2] + (1 << 13)) >> 14;
            out |= (uint32_t)v << (8 * j);
        }
    }
    uint8_t* d = dst + (size_t)y * dstride + x0;
    for (int j = 0; j < nx; ++j) d[j] = (uint8_t)(out >> (8 * j));
}

// Device staging of the host-array entry points: a pool of (device, non-blocking stream,
// growable buffer) slots taken for the length of one call.  After warm-up a call allocates
// nothing, and it waits only for its own stream, never for the device (the reference calls
// these from the Tracking thread while LocalMapping / LoopClosing run matchers).
struct Scratch {
    int device = -1;
    hipStream_t st = nullptr;
    DevBuf buf;
};
std::mutex g_scratch_mu;
std::vector<Scratch*> g_scratch_free;

struct ScratchLease {
    Scratch* s = nullptr;
    explicit ScratchLease(int device) {
        {
            std::lock_guard<std::mutex> lk(g_scratch_mu);
            for (size_t i = 0; i < g_scratch_free.size(); ++i)
                if (g_scratch_free[i]->device == device) {
                    s = g_scratch_free[i];
                    g_scratch_free.erase(g_scratch_free.begin() + i);
                    break;
                }
        }
        if (!s) {
            Scratch* n = new Scratch();
            n->device = device;
            if (!HIPOK(hipStreamCreateWithFlags(&n->st, hipStreamNonBlocking))) {
                delete n;
                return;
            }
            s = n;
        }
    }
    ~ScratchLease() {
        if (!s) return;
        std::lock_guard<std::mutex> lk(g_scratch_mu);
        g_scratch_free.push_back(s);   // slots live for the process (no teardown-order hazards)
    }
};

}  // namespace

extern "C" {

orbx_status orbx_cvt_color_device(const uint8_t* d_src, int32_t width, int32_t height,
                                  size_t src_stride, int32_t channels, int32_t rgb,
                                  uint8_t* d_dst, size_t dst_stride, void* stream) {
    if (width < 0 || height < 0 || (channels != 3 && channels != 4)) return ORBX_ERR_INVALID;
    if (width == 0 || height == 0) return ORBX_OK;
    if (!d_src || !d_dst || src_stride < (size_t)width * channels || dst_stride < (size_t)width)
        return ORBX_ERR_INVALID;
    hipLaunchKernelGGL(k_gray, dim3((width + 1023) / 1024, height), dim3(256), 0,
                       (hipStream_t)stream, d_src, width, height, src_stride, channels, rgb,
                       d_dst, dst_stride);
    return HIPOK(hipGetLastError()) ? ORBX_OK : ORBX_ERR_DEVICE;
}

orbx_status orbx_cvt_color(const uint8_t* src, int32_t width, int32_t height, size_t src_stride,
                           int32_t channels, int32_t rgb, uint8_t* dst, size_t dst_stride,
                           int device) {
    if (width < 0 || height < 0 || (channels != 3 && channels != 4)) return ORBX_ERR_INVALID;
    if (width == 0 || height == 0) return ORBX_OK;
    if (!src || !dst || src_stride < (size_t)width * channels || dst_stride < (size_t)width)
        return ORBX_ERR_INVALID;
    if (!HIPOK(hipSetDevice(device))) return ORBX_ERR_DEVICE;
    const size_t sb = (size_t)width * channels * height, db = (size_t)width * height;
    ScratchLease L(device);
    if (!L.s || !L.s->buf.ensure(sb + db)) return ORBX_ERR_DEVICE;
    hipStream_t st = L.s->st;
    uint8_t* ds = L.s->buf.as<uint8_t>();
    orbx_status s = ORBX_OK;
    if (!HIPOK(hipMemcpy2DAsync(ds, (size_t)width * channels, src, src_stride,
                                (size_t)width * channels, height, hipMemcpyHostToDevice, st)))
        s = ORBX_ERR_DEVICE;
    if (s == ORBX_OK)
        s = orbx_cvt_color_device(ds, width, height, (size_t)width * channels, channels, rgb,
                                  ds + sb, width, st);
    if (s == ORBX_OK && !HIPOK(hipMemcpy2DAsync(dst, dst_stride, ds + sb, width, width, height,
                                                hipMemcpyDeviceToHost, st)))
        s = ORBX_ERR_DEVICE;
    if (!HIPOK(hipStreamSynchronize(st))) s = ORBX_ERR_DEVICE;
    return s;
}

orbx_status orbx_undistort_keypoints_device(const float* K4, const float* dist, int32_t ndist,
                                            const orbx_keypoint* d_kps, int32_t n,
                                            orbx_keypoint* d_kps_un, void* stream) {
    UndistParams P;
    if (!make_params(K4, dist, ndist, P) || n < 0 || (n > 0 && (!d_kps || !d_kps_un)))
        return ORBX_ERR_INVALID;
    if (n == 0) return ORBX_OK;
    const int copy = dist[0] == 0.0f;   // Frame.cc:431: mvKeysUn = mvKeys
    hipLaunchKernelGGL(k_undistort, dim3((n + 255) / 256), dim3(256), 0, (hipStream_t)stream, P,
                       d_kps, n, d_kps_un, copy);
    return HIPOK(hipGetLastError()) ? ORBX_OK : ORBX_ERR_DEVICE;
}

orbx_status orbx_undistort_keypoints(const float* K4, const float* dist, int32_t ndist,
                                     const orbx_keypoint* kps, int32_t n,
                                     orbx_keypoint* kps_un, int device) {
    UndistParams P;
    if (!make_params(K4, dist, ndist, P) || n < 0 || (n > 0 && (!kps || !kps_un)))
        return ORBX_ERR_INVALID;
    if (n == 0) return ORBX_OK;
    if (!HIPOK(hipSetDevice(device))) return ORBX_ERR_DEVICE;
    const size_t bytes = sizeof(orbx_keypoint) * (size_t)n;
    ScratchLease L(device);
    if (!L.s || !L.s->buf.ensure(bytes)) return ORBX_ERR_DEVICE;
    hipStream_t st = L.s->st;
    orbx_keypoint* d = L.s->buf.as<orbx_keypoint>();
    orbx_status s = ORBX_OK;
    if (!HIPOK(hipMemcpyAsync(d, kps, bytes, hipMemcpyHostToDevice, st))) s = ORBX_ERR_DEVICE;
    if (s == ORBX_OK) s = orbx_undistort_keypoints_device(K4, dist, ndist, d, n, d, st);
    if (s == ORBX_OK && !HIPOK(hipMemcpyAsync(kps_un, d, bytes, hipMemcpyDeviceToHost, st)))
        s = ORBX_ERR_DEVICE;
    if (!HIPOK(hipStreamSynchronize(st))) s = ORBX_ERR_DEVICE;
    return s;
}

orbx_status orbx_image_bounds(const float* K4, const float* dist, int32_t ndist, int32_t width,
                              int32_t height, float* bounds) {
    UndistParams P;
    if (!make_params(K4, dist, ndist, P) || !bounds || width <= 0 || height <= 0)
        return ORBX_ERR_INVALID;
    if (dist[0] != 0.0f) {   // Frame.cc:463-480
        const float cx[4] = {0.0f, (float)width, 0.0f, (float)width};
        const float cy[4] = {0.0f, 0.0f, (float)height, (float)height};
        float ux[4], uy[4];
        for (int i = 0; i < 4; ++i) undistort_pt(P, cx[i], cy[i], ux[i], uy[i]);
        bounds[0] = std::min(ux[0], ux[2]);
        bounds[1] = std::max(ux[1], ux[3]);
        bounds[2] = std::min(uy[0], uy[1]);
        bounds[3] = std::max(uy[2], uy[3]);
    } else {   // :482-487
        bounds[0] = 0.0f;
        bounds[1] = (float)width;
        bounds[2] = 0.0f;
        bounds[3] = (float)height;
    }
    return ORBX_OK;
}

orbx_status orbx_assign_grid_device(const orbx_keypoint* d_kps, int32_t n, int32_t cols,
                                    int32_t rows, float min_x, float min_y, float inv_w,
                                    float inv_h, int32_t* d_grid_off, int32_t* d_grid_feat,
                                    void* stream) {
    if (n < 0 || cols <= 0 || rows <= 0 || (long long)cols * rows > 16384 - 1024 ||
        !d_grid_off || (n > 0 && (!d_kps || !d_grid_feat)))
        return ORBX_ERR_INVALID;
    const size_t lds = 4 * ((size_t)cols * rows + 1024);   // <= 64 KB: no attribute needed
    hipLaunchKernelGGL(k_grid, dim3(1), dim3(1024), lds, (hipStream_t)stream, d_kps, n,
                       (const int32_t*)nullptr, n, cols, rows, min_x, min_y, inv_w, inv_h,
                       d_grid_off, d_grid_feat);
    return HIPOK(hipGetLastError()) ? ORBX_OK : ORBX_ERR_DEVICE;
}

orbx_status orbx_assign_grid_batch_device(const orbx_keypoint* d_kps, int32_t kp_stride,
                                          const int32_t* d_n, int32_t batch, int32_t cols,
                                          int32_t rows, float min_x, float min_y, float inv_w,
                                          float inv_h, int32_t* d_grid_off,
                                          int32_t* d_grid_feat, void* stream) {
    if (batch < 0 || kp_stride < 0 || cols <= 0 || rows <= 0 ||
        (long long)cols * rows > 16384 - 1024)
        return ORBX_ERR_INVALID;
    if (batch == 0) return ORBX_OK;
    if (!d_kps || !d_n || !d_grid_off || !d_grid_feat) return ORBX_ERR_INVALID;
    const size_t lds = 4 * ((size_t)cols * rows + 1024);
    hipLaunchKernelGGL(k_grid, dim3(batch), dim3(1024), lds, (hipStream_t)stream, d_kps, 0, d_n,
                       kp_stride, cols, rows, min_x, min_y, inv_w, inv_h, d_grid_off,
                       d_grid_feat);
    return HIPOK(hipGetLastError()) ? ORBX_OK : ORBX_ERR_DEVICE;
}

orbx_status orbx_undistort_keypoints_batch_device(const float* K4, const float* dist,
                                                  int32_t ndist, const orbx_keypoint* d_kps,
                                                  int32_t kp_stride, const int32_t* d_n,
                                                  int32_t batch, orbx_keypoint* d_kps_un,
                                                  void* stream) {
    UndistParams P;
    if (!make_params(K4, dist, ndist, P) || batch < 0 || kp_stride < 0) return ORBX_ERR_INVALID;
    if (batch == 0 || kp_stride == 0) return ORBX_OK;
    if (!d_kps || !d_n || !d_kps_un || batch > 65535) return ORBX_ERR_INVALID;
    const int copy = dist[0] == 0.0f;
    hipLaunchKernelGGL(k_undistort_batch, dim3((kp_stride + 255) / 256, batch), dim3(256), 0,
                       (hipStream_t)stream, P, d_kps, kp_stride, d_n, d_kps_un, copy);
    return HIPOK(hipGetLastError()) ? ORBX_OK : ORBX_ERR_DEVICE;
}

}  // extern "C"
