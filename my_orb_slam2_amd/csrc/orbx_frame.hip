// orbx_frame.hip — per-frame geometry around the matchers (include/orbx_frame.h).
//
//   k_undistort    one lane per keypoint: cvUndistortPoints (OpenCV 3.2) in double, the
//                  same __host__ __device__ routine the host uses for ComputeImageBounds
//   k_grid         Frame::AssignFeaturesToGrid as a counting sort, one workgroup per frame:
//                  cell of every keypoint (PosInGrid, std::round half away from zero in
//                  float), per-cell LDS counts, a block scan over the 3072 cells, an atomic
//                  fill, then each cell sorted by feature index (the push_back order)
//   k_frustum      one lane per (frame, local MapPoint): Frame::isInFrustum + PredictScale, the
//                  SearchByProjection query of every MapPoint in view (SearchLocalPoints)
#include <hip/hip_runtime.h>

#include <cmath>
#include <mutex>
#include <vector>

#include "../../include/orbx_frame.h"
#include "orbx_device.h"
#include "orbx_host.h"
#include "orbx_math.h"

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

// Frame::isInFrustum (src/Frame.cc:285-349) with MapPoint::PredictScale (MapPoint.cc:430-444)
// and the query SearchByProjection(Frame&, vpMapPoints, th) forms from its outputs
// (ORBmatcher.cc:55-80).  The float / double steps follow the reference's types (see
// include/orbx_frame.h); the library is built with -ffp-contract=off, so every float op is
// rounded on its own as on x86.
__device__ __forceinline__ bool frustum_query(const orbx_frame_pose& F, const orbx_map_point& M,
                                              float cos_lim, float th, orbx_proj_query& q) {
    // Pc = mRcw*P + mtcw: cv::gemm(Rcw, P, 1, tcw, 1) small-matrix path (len 3, one column):
    // t_r = a_r0*b0 + a_r1*b1 + a_r2*b2 in float, d_r = (float)(t_r*1.0 + c_r*1.0)
    float Pc[3];
#pragma unroll
    for (int r = 0; r < 3; ++r) {
        float t = __fmul_rn(F.Rcw[3 * r], M.pos[0]);
        t = __fadd_rn(t, __fmul_rn(F.Rcw[3 * r + 1], M.pos[1]));
        t = __fadd_rn(t, __fmul_rn(F.Rcw[3 * r + 2], M.pos[2]));
        Pc[r] = (float)((double)t + (double)F.tcw[r]);
    }
    if (Pc[2] < 0.0f) return false;                       // positive depth
    const float invz = __fdiv_rn(1.0f, Pc[2]);
    const float u = __fadd_rn(__fmul_rn(__fmul_rn(F.fx, Pc[0]), invz), F.cx);
    const float v = __fadd_rn(__fmul_rn(__fmul_rn(F.fy, Pc[1]), invz), F.cy);
    if (u < F.min_x || u > F.max_x) return false;
    if (v < F.min_y || v > F.max_y) return false;
    const float maxD = __fmul_rn(1.2f, M.max_dist), minD = __fmul_rn(0.8f, M.min_dist);
    // PO = P - mOw; dist = cv::norm(PO): squares accumulated in double (normL2Sqr<float,
    // double>), sqrt, stored in a float
    const float PO[3] = {__fsub_rn(M.pos[0], F.Ow[0]), __fsub_rn(M.pos[1], F.Ow[1]),
                         __fsub_rn(M.pos[2], F.Ow[2])};
    double ss = 0.0;
#pragma unroll
    for (int k = 0; k < 3; ++k) ss = __dadd_rn(ss, __dmul_rn((double)PO[k], (double)PO[k]));
    const float dist = (float)__dsqrt_rn(ss);
    if (dist < minD || dist > maxD) return false;
    // viewCos = PO.dot(Pn) / dist: Mat::dot in double (dotProd_), / dist in double
    double dot = 0.0;
#pragma unroll
    for (int k = 0; k < 3; ++k) dot = __dadd_rn(dot, __dmul_rn((double)PO[k], (double)M.normal[k]));
    const float viewCos = (float)__ddiv_rn(dot, (double)dist);
    if (viewCos < cos_lim) return false;
    // PredictScale: ceil(log(ratio) / mfLogScaleFactor) on floats (std::log / std::ceil)
    const float ratio = __fdiv_rn(M.max_dist, dist);
    const float qf = ceilf(__fdiv_rn(glibc_logf(ratio), F.log_scale_factor));
    // (int) of a float as x86 cvttss2si: INT_MIN when out of range or NaN
    int lvl = (qf >= -2147483648.0f && qf < 2147483648.0f) ? (int)qf : INT_MIN;
    if (lvl < 0) lvl = 0;
    else if (lvl >= F.nlevels) lvl = F.nlevels - 1;
    // SearchByProjection: r = RadiusByViewingCos (viewCos > 0.998 in double), * th if th != 1
    float r = (double)viewCos > 0.998 ? 2.5f : 4.0f;
    if ((double)th != 1.0) r = __fmul_rn(r, th);
    q.u = u;
    q.v = v;
    q.ur = __fsub_rn(u, __fmul_rn(F.mbf, invz));        // mTrackProjXR
    q.radius = __fmul_rn(r, F.scale[lvl]);
    q.min_level = lvl - 1;
    q.max_level = lvl;
    q.pred_level = lvl;
    q.angle = 0.0f;
    return true;
}

__global__ __launch_bounds__(256) void k_frustum(const orbx_frame_pose* __restrict__ frames,
                                                 const orbx_map_point* __restrict__ mps,
                                                 const int32_t* __restrict__ mp_off,
                                                 const uint8_t* __restrict__ skip, float cos_lim,
                                                 float th, orbx_proj_query* __restrict__ q,
                                                 int32_t* __restrict__ nvisible) {
    const int f = blockIdx.y;
    const int b = mp_off[f], e = mp_off[f + 1];
    const int i = b + blockIdx.x * 256 + threadIdx.x;
    bool vis = false;
    if (i < e) {
        orbx_proj_query out;
        vis = (!skip || !skip[i]) && frustum_query(frames[f], mps[i], cos_lim, th, out);
        if (!vis) {
            out.u = out.v = out.ur = 0.0f;
            out.radius = -1.0f;
            out.min_level = out.max_level = out.pred_level = -1;
            out.angle = 0.0f;
        }
        q[i] = out;
    }
    if (nvisible) {
        const uint64_t m = __ballot(vis);
        if ((threadIdx.x & 63) == 0 && m) atomicAdd(&nvisible[f], (int)__popcll(m));
    }
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

orbx_status orbx_is_in_frustum_batch_device(const orbx_frame_pose* d_frames, int32_t nframes,
                                            const orbx_map_point* d_mps,
                                            const int32_t* d_mp_off, int32_t max_mps,
                                            const uint8_t* d_skip, float viewing_cos_limit,
                                            float th, orbx_proj_query* d_q,
                                            int32_t* d_nvisible, void* stream) {
    if (nframes < 0 || max_mps < 0 || nframes > 65535) return ORBX_ERR_INVALID;
    if (nframes == 0) return ORBX_OK;
    if (!d_frames || !d_mp_off || (max_mps > 0 && (!d_mps || !d_q))) return ORBX_ERR_INVALID;
    hipStream_t st = (hipStream_t)stream;
    if (d_nvisible && !HIPOK(hipMemsetAsync(d_nvisible, 0, 4 * (size_t)nframes, st)))
        return ORBX_ERR_DEVICE;
    if (max_mps == 0) return ORBX_OK;
    hipLaunchKernelGGL(k_frustum, dim3((max_mps + 255) / 256, nframes), dim3(256), 0, st,
                       d_frames, d_mps, d_mp_off, d_skip, viewing_cos_limit, th, d_q, d_nvisible);
    return HIPOK(hipGetLastError()) ? ORBX_OK : ORBX_ERR_DEVICE;
}

orbx_status orbx_is_in_frustum(const orbx_frame_pose* frame, const orbx_map_point* mps,
                               int32_t n, const uint8_t* skip, float viewing_cos_limit,
                               float th, orbx_proj_query* q, int32_t* nvisible, int device) {
    if (!frame || n < 0 || (n > 0 && (!mps || !q)) || frame->nlevels < 1 || frame->nlevels > 16)
        return ORBX_ERR_INVALID;
    if (n == 0) {
        if (nvisible) *nvisible = 0;
        return ORBX_OK;
    }
    if (!HIPOK(hipSetDevice(device))) return ORBX_ERR_DEVICE;
    auto al = [](size_t v) { return (v + 255) & ~(size_t)255; };
    const size_t o_f = 0, o_off = al(sizeof(orbx_frame_pose)), o_cnt = o_off + 256,
                 o_mp = o_cnt + 256, o_sk = o_mp + al(sizeof(orbx_map_point) * (size_t)n),
                 o_q = o_sk + al((size_t)n), end = o_q + sizeof(orbx_proj_query) * (size_t)n;
    ScratchLease L(device);
    if (!L.s || !L.s->buf.ensure(end)) return ORBX_ERR_DEVICE;
    hipStream_t st = L.s->st;
    uint8_t* d = L.s->buf.as<uint8_t>();
    const int32_t off[2] = {0, n};
    int32_t cnt = 0;
    orbx_status s = ORBX_OK;
    if (!HIPOK(hipMemcpyAsync(d + o_f, frame, sizeof(*frame), hipMemcpyHostToDevice, st)) ||
        !HIPOK(hipMemcpyAsync(d + o_off, off, sizeof(off), hipMemcpyHostToDevice, st)) ||
        !HIPOK(hipMemcpyAsync(d + o_mp, mps, sizeof(orbx_map_point) * (size_t)n,
                              hipMemcpyHostToDevice, st)) ||
        (skip && !HIPOK(hipMemcpyAsync(d + o_sk, skip, (size_t)n, hipMemcpyHostToDevice, st))))
        s = ORBX_ERR_DEVICE;
    if (s == ORBX_OK)
        s = orbx_is_in_frustum_batch_device((const orbx_frame_pose*)(d + o_f), 1,
                                            (const orbx_map_point*)(d + o_mp),
                                            (const int32_t*)(d + o_off), n,
                                            skip ? d + o_sk : nullptr, viewing_cos_limit, th,
                                            (orbx_proj_query*)(d + o_q), (int32_t*)(d + o_cnt), st);
    if (s == ORBX_OK &&
        (!HIPOK(hipMemcpyAsync(q, d + o_q, sizeof(orbx_proj_query) * (size_t)n,
                               hipMemcpyDeviceToHost, st)) ||
         !HIPOK(hipMemcpyAsync(&cnt, d + o_cnt, 4, hipMemcpyDeviceToHost, st))))
        s = ORBX_ERR_DEVICE;
    if (!HIPOK(hipStreamSynchronize(st))) s = ORBX_ERR_DEVICE;
    if (s == ORBX_OK && nvisible) *nvisible = cnt;
    return s;
}

}  // extern "C"
