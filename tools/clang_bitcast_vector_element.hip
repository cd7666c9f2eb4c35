// Reproducer of a compiler defect met in k_orient_desc (ROCm 7.2 hipcc / clang, gfx950):
// __builtin_bit_cast of an ext_vector_type element (rc.y) yields element 0.  In the IR
// after SROA the second store reads `extractelement <2 x float> %v, i32 0` although the
// source says rc.y; the -O0 IR is correct.  Copying the element into a plain float first
// (`const float fy = rc.y; __builtin_bit_cast(uint32_t, fy)`) gives the right code.
// In round 2 this is what made the packed-f32 rBRIEF form produce different descriptors
// (DESIGN.md §9, 6.).
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -S --cuda-device-only tools/clang_bitcast_vector_element.hip
// `k_bad` stores the same register twice; `k_good` stores both lanes of one v_pk_add_f32.
#include <hip/hip_runtime.h>
#include <stdint.h>
typedef float f2v __attribute__((ext_vector_type(2)));

__global__ void k_bad(const float* in, uint32_t* o) {
    const float px = in[threadIdx.x], py = in[threadIdx.x + 64], sb = in[128], ca = in[129];
    const f2v rc = f2v{px, px} * f2v{sb, ca} + f2v{py, -py} * f2v{ca, sb};
    o[threadIdx.x] = __builtin_bit_cast(uint32_t, rc.x);
    o[threadIdx.x + 64] = __builtin_bit_cast(uint32_t, rc.y);     // miscompiled: rc.x
}

__global__ void k_good(const float* in, uint32_t* o) {
    const float px = in[threadIdx.x], py = in[threadIdx.x + 64], sb = in[128], ca = in[129];
    const f2v rc = f2v{px, px} * f2v{sb, ca} + f2v{py, -py} * f2v{ca, sb};
    const float fx = rc.x, fy = rc.y;
    o[threadIdx.x] = __builtin_bit_cast(uint32_t, fx);
    o[threadIdx.x + 64] = __builtin_bit_cast(uint32_t, fy);
}
