// launch_attr.cpp — per-device launch facts shared by every launch wrapper.
//
// hipFuncSetAttribute(MaxDynamicSharedMemorySize) and the occupancy answer
// belong to a (kernel, device) pair, and contexts on different devices may be
// driven from different host threads at once (one pq_ctx per
// device, one host thread each).  The wrappers used to keep them in
// function-local statics, set once per process on whichever device happened
// to be current; this table keys them by the current device and is guarded
// by a mutex.
#include <hip/hip_runtime.h>

#include <map>
#include <mutex>
#include <tuple>

#include "kernels/kernels.hpp"

namespace pqk {
namespace {

std::mutex g_mu;
std::map<std::pair<const void*, int>, uint32_t> g_lds;                 // (kernel, device) -> dynamic LDS limit set
std::map<std::tuple<const void*, int, int, uint32_t>, int> g_resident;  // (kernel, device, threads, LDS) -> blocks per CU
std::map<int, int> g_cus;                                             // device -> compute units

int current_device() {
    int d = 0;
    if (hipGetDevice(&d) != hipSuccess) d = 0;
    return d;
}

}  // namespace

bool ensure_dyn_lds(const void* fn, uint32_t bytes) {
    const int dev = current_device();
    std::lock_guard<std::mutex> lk(g_mu);
    uint32_t& have = g_lds[{fn, dev}];
    if (bytes <= have) return true;
    if (hipFuncSetAttribute(fn, hipFuncAttributeMaxDynamicSharedMemorySize, static_cast<int>(bytes)) != hipSuccess) {
        (void)hipGetLastError();  // clear the sticky error: the caller's launch check must not see it
        return false;
    }
    have = bytes;
    return true;
}

int resident_blocks(const void* fn, int threads, uint32_t lds) {
    const int dev = current_device();
    {
        std::lock_guard<std::mutex> lk(g_mu);
        auto it = g_resident.find({fn, dev, threads, lds});
        if (it != g_resident.end()) return it->second;
    }
    if (lds && !ensure_dyn_lds(fn, lds)) return 0;
    int occ = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&occ, fn, threads, lds) != hipSuccess || occ < 1) {
        (void)hipGetLastError();
        occ = 1;
    }
    std::lock_guard<std::mutex> lk(g_mu);
    g_resident[{fn, dev, threads, lds}] = occ;
    return occ;
}

int device_cus() {
    const int dev = current_device();
    {
        std::lock_guard<std::mutex> lk(g_mu);
        auto it = g_cus.find(dev);
        if (it != g_cus.end()) return it->second;
    }
    int cus = 0;
    if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus < 1) cus = 256;
    std::lock_guard<std::mutex> lk(g_mu);
    g_cus[dev] = cus;
    return cus;
}

}  // namespace pqk
