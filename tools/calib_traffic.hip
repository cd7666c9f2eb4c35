// Calibration of the rocprofv3 FETCH_SIZE / WRITE_SIZE counters for the access widths and
// patterns the extraction kernels use (MI355X_MICROARCH.md §HBM: only 16-byte-per-lane
// streams are calibrated there; "calibrate on a known byte count in your own access
// pattern").  Every kernel below moves a known number of distinct bytes over a KITTI-size
// level-0 batch (1024 images x 376 rows, 1280-byte pitch, 1241 bytes used per row):
//
//   k_lin_d4      dword per lane, fully coalesced copy of the whole padded batch
//   k_lin_d16     16 bytes per lane, the same copy (the guide's calibrated width)
//   k_strip       the k_level_strip<4> geometry: a wave = two half-strips of 30 interior
//                 lanes (120 bytes) + one halo lane per side, 64 output rows per strip read
//                 with 3 halo rows above and below, dword loads, interior dword stores
//   k_strip_core  the same walk without halo rows or halo lanes (reads = writes = image)
//   k_strip_buf   k_strip with k_level_strip's stores: raw buffer stores on every step, the
//                 halo lanes and halo rows dropped by an offset past num_records
//   k_rows128     whole 128-byte row segments per half-wave (32 lanes), no halos
//
// Each prints nothing but its launch; the byte counts to compare against are printed once.
// hipcc --offload-arch=gfx950 -O3 tools/calib_traffic.hip -o tools/_build/calib_traffic
// rocprofv3 --pmc FETCH_SIZE -- tools/_build/calib_traffic   (WRITE_SIZE in its own pass)
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

#define NIMG 1024
#define H 376
#define W 1241
#define PITCH 1280
#define STH 64
#define HALF 30                         // interior lanes per half-strip (4 bytes each)
#define NHALF ((W / 4 + HALF - 1) / HALF)   // 11 half-strips per row
#define NWAVE ((NHALF + 1) / 2)             // 6 waves per row strip
#define NSTRIP ((H + STH - 1) / STH)        // 6 row strips

static const size_t IMG = (size_t)H * PITCH;

__global__ void k_lin_d4(const uint32_t* __restrict__ s, uint32_t* __restrict__ d, size_t n) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) d[i] = s[i] + 1u;
}

__global__ void k_lin_d16(const uint4* __restrict__ s, uint4* __restrict__ d, size_t n) {
    size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) { uint4 v = s[i]; v.x += 1u; d[i] = v; }
}

// one wave per (image, strip, wave index); 4 waves per block
template <bool HALO>
__global__ void k_strip(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst) {
    const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63, half = lane >> 5, l32 = lane & 31;
    const int img = blockIdx.y;
    const int strip = wave / NWAVE, w = wave - strip * NWAVE;
    if (strip >= NSTRIP) return;
    const int hs = 2 * w + half;
    const int g = HALF * hs + (l32 - 1);           // group index of this lane (halo: -1 / 30)
    const bool interior = l32 >= 1 && l32 <= HALF && 4 * g < W && hs < NHALF;
    const bool reads = HALO ? (g >= 0 && 4 * g < PITCH && hs < NHALF && l32 <= HALF + 1) : interior;
    const int r0 = strip * STH, r1 = min(r0 + STH, H);
    const int a0 = HALO ? max(r0 - 3, 0) : r0, a1 = HALO ? min(r1 + 3, H) : r1;
    const uint8_t* sp = src + (size_t)img * IMG + 4 * g;
    uint8_t* dp = dst + (size_t)img * IMG + 4 * g;
    uint32_t acc = 0;
    for (int r = a0; r < a1; ++r) {
        const uint32_t v = reads ? *(const uint32_t*)(sp + (size_t)r * PITCH) : 0u;
        acc = acc * 3u + v;
        if (interior && r >= r0 && r < r1)
            *(uint32_t*)(dp + (size_t)r * PITCH) = acc;
    }
}

// k_strip<true> with the stores of k_level_strip (STRIP_BUFST): every lane stores every step
// by a raw buffer store, a lane or step with nothing to write getting an offset past
// num_records (dropped by the range check)
__global__ void k_strip_buf(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst) {
    const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63, half = lane >> 5, l32 = lane & 31;
    const int img = blockIdx.y;
    const int strip = wave / NWAVE, w = wave - strip * NWAVE;
    if (strip >= NSTRIP) return;
    const int hs = 2 * w + half;
    const int g = HALF * hs + (l32 - 1);
    const bool interior = l32 >= 1 && l32 <= HALF && 4 * g < W && hs < NHALF;
    const bool reads = g >= 0 && 4 * g < PITCH && hs < NHALF && l32 <= HALF + 1;
    const int r0 = strip * STH, r1 = min(r0 + STH, H);
    const int a0 = max(r0 - 3, 0), a1 = min(r1 + 3, H);
    const uint8_t* sp = src + (size_t)img * IMG + 4 * g;
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(dst + (size_t)img * IMG, 0, H * PITCH, 0x00020000);
    const uint32_t lane_off = interior ? (uint32_t)(4 * g) : 0x80000000u;
    uint32_t acc = 0;
    for (int r = a0; r < a1; ++r) {
        const uint32_t v = reads ? *(const uint32_t*)(sp + (size_t)r * PITCH) : 0u;
        acc = acc * 3u + v;
        const bool ok = r >= r0 && r < r1;
        __builtin_amdgcn_raw_buffer_store_b32(acc, rs, ok ? lane_off : 0x80000000u, ok ? r * PITCH : 0, 0);
    }
}

// half-wave writes / reads 128 aligned bytes per row (32 lanes x 4 B), no halos
__global__ void k_rows128(const uint8_t* __restrict__ src, uint8_t* __restrict__ dst) {
    const int wave = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int lane = threadIdx.x & 63, half = lane >> 5, l32 = lane & 31;
    const int img = blockIdx.y;
    const int seg = PITCH / 128;                  // 10 segments per row
    const int strip = wave / (seg / 2), w = wave - strip * (seg / 2);
    if (strip >= NSTRIP) return;
    const int col = 128 * (2 * w + half) + 4 * l32;
    const int r0 = strip * STH, r1 = min(r0 + STH, H);
    const uint8_t* sp = src + (size_t)img * IMG + col;
    uint8_t* dp = dst + (size_t)img * IMG + col;
    uint32_t acc = 0;
    for (int r = r0; r < r1; ++r) {
        acc = acc * 3u + *(const uint32_t*)(sp + (size_t)r * PITCH);
        *(uint32_t*)(dp + (size_t)r * PITCH) = acc;
    }
}

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { \
    fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_)); return 1; } } while (0)

int main() {
    const size_t bytes = (size_t)NIMG * IMG;
    uint8_t *a, *b;
    CK(hipMalloc(&a, bytes));
    CK(hipMalloc(&b, bytes));
    CK(hipMemset(a, 7, bytes));
    CK(hipMemset(b, 0, bytes));
    // an unrelated 512 MB write between kernels evicts the 256 MB Infinity Cache
    uint8_t* flush;
    const size_t fl = 512ull << 20;
    CK(hipMalloc(&flush, fl));
    auto evict = [&]() { return hipMemset(flush, 1, fl); };
    const size_t ndw = bytes / 4, n16 = bytes / 16;
    // distinct bytes of the strip patterns
    const size_t used_row = (size_t)((W + 3) / 4) * 4;           // 1244: whole groups
    const size_t core = (size_t)NIMG * H * used_row;
    printf("bytes padded batch      %zu\n", bytes);
    printf("bytes strip interior    %zu (1241 bytes rounded to whole 4-byte groups per row)\n", core);
    for (int rep = 0; rep < 2; ++rep) {
        CK(evict());
        hipLaunchKernelGGL(k_lin_d4, dim3((ndw + 255) / 256), dim3(256), 0, 0, (const uint32_t*)a, (uint32_t*)b, ndw);
        CK(evict());
        hipLaunchKernelGGL(k_lin_d16, dim3((n16 + 255) / 256), dim3(256), 0, 0, (const uint4*)a, (uint4*)b, n16);
        CK(evict());
        hipLaunchKernelGGL(k_strip<true>, dim3((NSTRIP * NWAVE + 3) / 4, NIMG), dim3(256), 0, 0, a, b);
        CK(evict());
        hipLaunchKernelGGL(k_strip<false>, dim3((NSTRIP * NWAVE + 3) / 4, NIMG), dim3(256), 0, 0, a, b);
        CK(evict());
        hipLaunchKernelGGL(k_strip_buf, dim3((NSTRIP * NWAVE + 3) / 4, NIMG), dim3(256), 0, 0, a, b);
        CK(evict());
        hipLaunchKernelGGL(k_rows128, dim3((NSTRIP * (PITCH / 256) + 3) / 4, NIMG), dim3(256), 0, 0, a, b);
        CK(hipDeviceSynchronize());
    }
    CK(hipFree(a));
    CK(hipFree(b));
    CK(hipFree(flush));
    printf("done\n");
    return 0;
}
