// calib_fetch.hip -- FETCH_SIZE / WRITE_SIZE calibration for the access
// widths the dpg kernels use (MI355X_MICROARCH.md: FETCH_SIZE is exact only
// for 16-B/lane streaming loads after doubling; other widths are
// uncalibrated).  Each kernel moves a known number of bytes; run under
//   rocprofv3 --pmc FETCH_SIZE -- ./calib_fetch     (and WRITE_SIZE)
// and divide.  Build: hipcc --offload-arch=gfx950 -O3 -o calib_fetch calib_fetch.hip
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <vector>

// coalesced streaming read, 8 B per lane
__global__ void k_read8(const uint64_t *a, size_t n, uint64_t *out) {
    uint64_t s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x)
        s ^= a[i];
    if (s == 0x123456789ull) out[0] = s;  // keep the loads
}

// coalesced streaming read, 16 B per lane
__global__ void k_read16(const uint4 *a, size_t n, uint64_t *out) {
    uint32_t s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x) {
        const uint4 v = a[i];
        s ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (s == 0x12345u) out[0] = s;
}

// random 8-B gathers (one per lane, distinct 64-B sectors)
__global__ void k_gather8(const uint64_t *a, size_t n_sectors, size_t n_reads, uint64_t *out) {
    uint64_t s = 0;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n_reads;
         i += (size_t)gridDim.x * blockDim.x) {
        const size_t sec = (i * 0x9E3779B97F4A7C15ull >> 20) % n_sectors;
        s ^= a[sec * 8];
    }
    if (s == 0x123456789ull) out[0] = s;
}

// coalesced streaming write, 8 B per lane
__global__ void k_write8(uint64_t *a, size_t n) {
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n;
         i += (size_t)gridDim.x * blockDim.x)
        a[i] = i;
}

int main() {
    const size_t bytes = (size_t)4 << 30;  // 4 GiB: far beyond the 256 MiB Infinity Cache
    uint64_t *a = nullptr, *out = nullptr;
    if (hipMalloc(&a, bytes) != hipSuccess || hipMalloc(&out, 64) != hipSuccess) return 1;
    (void)hipMemset(a, 1, bytes);
    const size_t n8 = bytes / 8;
    const size_t n_reads = (size_t)1 << 26;  // 64 Mi gathers
    // the second repetition is timed: a gather's true HBM cost shows in its
    // rate against the streaming read's (both far beyond the caches)
    hipEvent_t ev[5];
    for (auto &e : ev) (void)hipEventCreate(&e);
    for (int rep = 0; rep < 2; ++rep) {
        (void)hipEventRecord(ev[0]);
        k_read8<<<4096, 256>>>(a, n8, out);
        (void)hipEventRecord(ev[1]);
        k_read16<<<4096, 256>>>(reinterpret_cast<const uint4 *>(a), bytes / 16, out);
        (void)hipEventRecord(ev[2]);
        k_gather8<<<4096, 256>>>(a, bytes / 64, n_reads, out);
        (void)hipEventRecord(ev[3]);
        k_write8<<<4096, 256>>>(a, n8);
        (void)hipEventRecord(ev[4]);
    }
    (void)hipDeviceSynchronize();
    float ms[4];
    for (int i = 0; i < 4; ++i) (void)hipEventElapsedTime(&ms[i], ev[i], ev[i + 1]);
    std::printf("{\"read_bytes\": %zu, \"gather_reads\": %zu, \"write_bytes\": %zu, "
                "\"ms\": {\"k_read8\": %.4f, \"k_read16\": %.4f, \"k_gather8\": %.4f, "
                "\"k_write8\": %.4f}}\n",
                bytes, n_reads, bytes, ms[0], ms[1], ms[2], ms[3]);
    return 0;
}
