// Known-bytes kernels for calibrating rocprofv3's FETCH_SIZE / WRITE_SIZE on
// gfx950 at the access widths the ORB kernels use (MI355X_MICROARCH.md §HBM:
// only 16 B/lane streaming reads and writes are calibrated there).  Each kernel
// streams exactly kBytes through one access width; the buffers are 1 GiB each
// (4x the 256 MiB Infinity Cache) and touched round-robin, so no kernel's data
// is cache-resident from the previous one.  Prints one JSON line per kernel
// with its algorithmic byte count; tools/pmc_calibrate.py divides the counter
// readings by it.  Build: hipcc --offload-arch=gfx950 -O3 (tools/calib/build.sh).
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr size_t kBytes = size_t(1) << 30;
constexpr int kNT = 256;

#define CHECK(x)                                                                          \
    do {                                                                                  \
        hipError_t e = (x);                                                               \
        if (e != hipSuccess) {                                                            \
            fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                        \
            return 1;                                                                     \
        }                                                                                 \
    } while (0)

// one dword per lane, buffer loads (FAST strip / blur / resize use raw_buffer_load_b32)
__global__ __launch_bounds__(kNT) void calib_read_b32_buffer(const uint8_t* src, uint32_t* sink) {
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(src), 0, 0x7FFFFFFF, 0x00020000);
    uint32_t acc = 0;
    const size_t per_block = kBytes / gridDim.x;  // multiple of 4 KiB
    const uint32_t base = (uint32_t)(blockIdx.x * per_block);
    for (uint32_t off = threadIdx.x * 4; off < per_block; off += kNT * 4)
        acc ^= (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rsrc, off, base, 0);
    if (acc == 0x12345678u) sink[blockIdx.x] = acc;  // keeps the loads; never true for memset data
}

__global__ __launch_bounds__(kNT) void calib_read_b128_global(const uint4* src, uint32_t* sink) {
    uint32_t acc = 0;
    const size_t n = kBytes / 16;
    for (size_t i = blockIdx.x * (size_t)kNT + threadIdx.x; i < n; i += (size_t)gridDim.x * kNT) {
        const uint4 v = src[i];
        acc ^= v.x ^ v.y ^ v.z ^ v.w;
    }
    if (acc == 0x12345678u) sink[blockIdx.x] = acc;
}

// (acc stays below 256, so the sink test must be a byte value or the compiler drops the loads:
// round 2's b8 reading of 4 KB per GiB was that)
__global__ __launch_bounds__(kNT) void calib_read_b8_global(const uint8_t* src, uint32_t* sink) {
    uint32_t acc = 0;
    for (size_t i = blockIdx.x * (size_t)kNT + threadIdx.x; i < kBytes; i += (size_t)gridDim.x * kNT) acc ^= src[i];
    if (acc == 0x5Au) sink[blockIdx.x] = acc;
}

__global__ __launch_bounds__(kNT) void calib_read_b32_global(const uint32_t* src, uint32_t* sink) {
    uint32_t acc = 0;
    const size_t n = kBytes / 4;
    for (size_t i = blockIdx.x * (size_t)kNT + threadIdx.x; i < n; i += (size_t)gridDim.x * kNT) acc ^= src[i];
    if (acc == 0x12345678u) sink[blockIdx.x] = acc;
}

__global__ __launch_bounds__(kNT) void calib_read_b64_global(const uint2* src, uint32_t* sink) {
    uint32_t acc = 0;
    const size_t n = kBytes / 8;
    for (size_t i = blockIdx.x * (size_t)kNT + threadIdx.x; i < n; i += (size_t)gridDim.x * kNT) {
        const uint2 v = src[i];
        acc ^= v.x ^ v.y;
    }
    if (acc == 0x12345678u) sink[blockIdx.x] = acc;
}

__global__ __launch_bounds__(kNT) void calib_write_b32_buffer(uint8_t* dst) {
    const auto rsrc = __builtin_amdgcn_make_buffer_rsrc(dst, 0, 0x7FFFFFFF, 0x00020000);
    const size_t per_block = kBytes / gridDim.x;
    const uint32_t base = (uint32_t)(blockIdx.x * per_block);
    for (uint32_t off = threadIdx.x * 4; off < per_block; off += kNT * 4)
        __builtin_amdgcn_raw_buffer_store_b32((int)(off ^ 0x5A5A5A5A), rsrc, off, base, 0);
}

__global__ __launch_bounds__(kNT) void calib_write_b32_global(uint32_t* dst) {
    const size_t n = kBytes / 4;
    for (size_t i = blockIdx.x * (size_t)kNT + threadIdx.x; i < n; i += (size_t)gridDim.x * kNT) dst[i] = (uint32_t)i;
}

__global__ __launch_bounds__(kNT) void calib_write_b128_global(uint4* dst) {
    const size_t n = kBytes / 16;
    for (size_t i = blockIdx.x * (size_t)kNT + threadIdx.x; i < n; i += (size_t)gridDim.x * kNT)
        dst[i] = make_uint4((uint32_t)i, 1u, 2u, 3u);
}

__global__ __launch_bounds__(kNT) void calib_write_b8_global(uint8_t* dst) {
    for (size_t i = blockIdx.x * (size_t)kNT + threadIdx.x; i < kBytes; i += (size_t)gridDim.x * kNT)
        dst[i] = (uint8_t)i;
}

int main() {
    uint8_t* buf[3];
    uint32_t* sink;
    for (auto& b : buf) CHECK(hipMalloc(&b, kBytes));
    CHECK(hipMalloc(&sink, 1 << 20));
    for (auto& b : buf) CHECK(hipMemset(b, 0x11, kBytes));
    CHECK(hipDeviceSynchronize());
    const int grid = 4096;  // kBytes / grid = 256 KiB per block
    // round-robin over the three buffers: each kernel's data was last touched two kernels ago (>= 1 GiB later)
    hipLaunchKernelGGL(calib_read_b32_buffer, dim3(grid), dim3(kNT), 0, 0, buf[0], sink);
    hipLaunchKernelGGL(calib_read_b128_global, dim3(grid), dim3(kNT), 0, 0, (const uint4*)buf[1], sink);
    hipLaunchKernelGGL(calib_read_b8_global, dim3(grid), dim3(kNT), 0, 0, buf[2], sink);
    hipLaunchKernelGGL(calib_write_b32_buffer, dim3(grid), dim3(kNT), 0, 0, buf[0]);
    hipLaunchKernelGGL(calib_write_b128_global, dim3(grid), dim3(kNT), 0, 0, (uint4*)buf[1]);
    hipLaunchKernelGGL(calib_write_b8_global, dim3(grid), dim3(kNT), 0, 0, buf[2]);
    hipLaunchKernelGGL(calib_write_b32_global, dim3(grid), dim3(kNT), 0, 0, (uint32_t*)buf[0]);
    hipLaunchKernelGGL(calib_read_b32_global, dim3(grid), dim3(kNT), 0, 0, (const uint32_t*)buf[1], sink);
    hipLaunchKernelGGL(calib_read_b64_global, dim3(grid), dim3(kNT), 0, 0, (const uint2*)buf[2], sink);
    CHECK(hipGetLastError());
    CHECK(hipDeviceSynchronize());
    const char* names[] = {"calib_read_b32_buffer",  "calib_read_b128_global",  "calib_read_b8_global",
                           "calib_write_b32_buffer", "calib_write_b128_global", "calib_write_b8_global",
                           "calib_write_b32_global", "calib_read_b32_global",   "calib_read_b64_global"};
    for (int i = 0; i < 9; ++i)
        printf("{\"kernel\": \"%s\", \"%s_bytes\": %zu}\n", names[i], names[i][6] == 'r' ? "read" : "write",
               kBytes);
    for (auto& b : buf) CHECK(hipFree(b));
    CHECK(hipFree(sink));
    return 0;
}
