// orbx_host.h — host-side helpers shared by the C-ABI translation units.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>

#define ORBX_MAX_DEVICES 64  // per-device kernel attribute caches (prepare_kernels, kfdb)

namespace orbx {

// Text of the first failing HIP call on this thread (orbx_last_error()).
extern thread_local char g_err[256];
// Records a failing HIP call into g_err; returns e == hipSuccess.
bool hip_ok(hipError_t e, const char* what);
#define HIPOK(call) ::orbx::hip_ok((call), #call)

// A growable device allocation (contents are not preserved across growth), or a view of
// part of another one (view(): never freed through this object).
struct DevBuf {
    void* p = nullptr;
    size_t n = 0;
    bool own = true;
    void release() {
        if (p && own) (void)hipFree(p);
        p = nullptr;
        n = 0;
        own = true;
    }
    void view(void* base, size_t bytes) {
        release();
        p = base;
        n = bytes;
        own = false;
    }
    bool ensure(size_t bytes) {
        if (bytes <= n && p && own) return true;
        release();
        if (bytes == 0) bytes = 16;
        if (!HIPOK(hipMalloc(&p, bytes))) { p = nullptr; return false; }
        n = bytes;
        return true;
    }
    template <class T> T* as() const { return (T*)p; }
};

}  // namespace orbx
