// orbx_kernels.h — host-side launch descriptors of the gfx950 kernels.
#pragma once
#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include "orbx_internal.h"

namespace orbx {

struct ExtractLaunch {
    const Geometry* hg;        // host copy of the geometry
    const Geometry* dg;        // device copy
    const CellDesc* cells;     // device
    const int16_t* rtab;       // device
    const uint8_t* d_imgs;
    size_t stride, batch_stride;
    int batch;
    uint8_t* pyr;
    uint8_t* blur;
    int* ccnt;
    uint32_t* cand;
    int* ocnt;
    uint32_t* okp;
    uint8_t* kscratch;
    long long kscratch_per_image;
    int ncap, kcap;
    size_t octree_lds;
    float* kps;
    uint8_t* desc;
    int* nkp;
};

struct StereoLaunch {
    const Geometry* dg;
    int batch;
    const float* kpsL;
    const uint8_t* descL;
    const int* nkpL;
    const uint8_t* pyrL;
    const float* kpsR;
    const uint8_t* descR;
    const int* nkpR;
    const uint8_t* pyrR;
    float mbf, mb;
    float* uR;
    float* depth;
    int* nvalid;
    size_t lds;
};

hipError_t launch_extract(const ExtractLaunch& a, hipStream_t st);
size_t octree_lds_bytes(int ncap, int kcap);
hipError_t launch_stereo(const StereoLaunch& a, hipStream_t st);
size_t stereo_lds_bytes(int kp_cap, int height);

}  // namespace orbx
