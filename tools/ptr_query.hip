// Which HIP pointer queries work on pinned host memory (hipHostMalloc, hipHostRegister) on this
// ROCm, at the allocation base and inside it?  pinned_view (merkle_capi.hip) needs the pinned
// range around a chunk and its device address.
// Build: hipcc --offload-arch=gfx950 -O2 -o tools/ptr_query tools/ptr_query.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

static void query(const char* what, void* p) {
    hipPointerAttribute_t a{};
    hipError_t e1 = hipPointerGetAttributes(&a, p);
    void* start = nullptr;
    size_t size = 0;
    hipError_t e2 = hipPointerGetAttribute(&start, HIP_POINTER_ATTRIBUTE_RANGE_START_ADDR, (hipDeviceptr_t)p);
    hipError_t e3 = hipPointerGetAttribute(&size, HIP_POINTER_ATTRIBUTE_RANGE_SIZE, (hipDeviceptr_t)p);
    size_t isz = 0;
    hipError_t e4 = hipMemPtrGetInfo(p, &isz);
    hipDeviceptr_t base = nullptr;
    size_t asz = 0;
    hipError_t e5 = hipMemGetAddressRange(&base, &asz, (hipDeviceptr_t)p);
    void* dp = nullptr;
    hipError_t e6 = hipHostGetDevicePointer(&dp, p, 0);
    (void)hipGetLastError();
    std::printf("%-28s p=%p | attrs rc=%d type=%d dev=%p host=%p | range rc=%d/%d start=%p size=%zu | "
                "MemPtrGetInfo rc=%d size=%zu | GetAddressRange rc=%d base=%p size=%zu | HostGetDevicePointer rc=%d %p\n",
                what, p, (int)e1, (int)a.type, a.devicePointer, a.hostPointer, (int)e2, (int)e3, start, size, (int)e4, isz,
                (int)e5, (void*)base, asz, (int)e6, dp);
}

int main() {
    const size_t n = 64 << 20;
    void* hm = nullptr;
    if (hipHostMalloc(&hm, n, hipHostMallocDefault) != hipSuccess) return 1;
    query("hipHostMalloc base", hm);
    query("hipHostMalloc +12345", (char*)hm + 12345);
    query("hipHostMalloc last byte", (char*)hm + n - 1);
    void* rg = std::aligned_alloc(4096, n);
    if (hipHostRegister(rg, n, hipHostRegisterDefault) != hipSuccess) return 2;
    query("hipHostRegister base", rg);
    query("hipHostRegister +12345", (char*)rg + 12345);
    query("hipHostRegister last byte", (char*)rg + n - 1);
    void* pg = std::malloc(n);
    query("pageable malloc", pg);
    void* dv = nullptr;
    if (hipMalloc(&dv, n) != hipSuccess) return 3;
    query("hipMalloc +12345", (char*)dv + 12345);
    (void)hipHostUnregister(rg);
    (void)hipHostFree(hm);
    (void)hipFree(dv);
    std::free(rg);
    std::free(pg);
    return 0;
}
