// Calibration of rocprofv3's FETCH_SIZE / WRITE_SIZE on gfx950 for the access widths the
// table build and the forward use (MI355X_MICROARCH.md § HBM: only 16-B-per-lane streaming
// reads are calibrated there — FETCH_SIZE reports half of their bytes).  Each kernel streams a
// known byte count once (buffers of 512 MB: past the 256 MB Infinity Cache), one launch each,
// in a fixed order; the PMC passes attribute counters per dispatch.
//
//   hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o tools/fetch_calib
//   rocprofv3 --pmc FETCH_SIZE -d DIR -o calib --output-format csv -- tools/fetch_calib
//   rocprofv3 --pmc WRITE_SIZE -d DIR -o calib --output-format csv -- tools/fetch_calib
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>

constexpr int64_t kBytes = 512ll << 20;

template <typename T>
__global__ void read_kernel(const T* __restrict__ a, int64_t n, float* __restrict__ sink) {
    float acc = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x) {
        const T v = a[i];
        const uint32_t* w = reinterpret_cast<const uint32_t*>(&v);
        for (int k = 0; k < (int)(sizeof(T) / 4); ++k) acc += __uint_as_float(w[k]);
        if constexpr (sizeof(T) < 4) acc += (float)*reinterpret_cast<const uint16_t*>(&v);
    }
    if (acc == 1.2345f) sink[0] = acc;   // (never: keeps the loads)
}

template <typename T>
__global__ void write_kernel(T* __restrict__ a, int64_t n) {
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        a[i] = T{};
}

// the table build's staged gather: 4 + 8 B per segment, striped over the lanes
__global__ void read_pair_kernel(const int32_t* __restrict__ v, const double* __restrict__ l,
                                 int64_t n, float* __restrict__ sink) {
    float acc = 0.f;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (int64_t)gridDim.x * blockDim.x)
        acc += (float)v[i] + (float)l[i];
    if (acc == 1.2345f) sink[0] = acc;
}

int main() {
    void* buf;
    void* buf2;
    float* sink;
    if (hipMalloc(&buf, kBytes) != hipSuccess || hipMalloc(&buf2, kBytes) != hipSuccess ||
        hipMalloc(&sink, 64) != hipSuccess)
        return 1;
    hipMemset(buf, 0, kBytes);
    hipMemset(buf2, 0, kBytes);
    const dim3 g(256 * 32), b(256);
    // dispatch order (the records name them by kernel): reads 2 / 4 / 8 / 16 B per lane, the
    // 4 + 8 B pair, writes 2 / 4 / 8 / 16 B per lane
    hipLaunchKernelGGL(read_kernel<uint16_t>, g, b, 0, 0, (const uint16_t*)buf, kBytes / 2, sink);
    hipLaunchKernelGGL(read_kernel<uint32_t>, g, b, 0, 0, (const uint32_t*)buf, kBytes / 4, sink);
    hipLaunchKernelGGL(read_kernel<uint2>, g, b, 0, 0, (const uint2*)buf, kBytes / 8, sink);
    hipLaunchKernelGGL(read_kernel<uint4>, g, b, 0, 0, (const uint4*)buf, kBytes / 16, sink);
    hipLaunchKernelGGL(read_pair_kernel, g, b, 0, 0, (const int32_t*)buf, (const double*)buf2,
                       kBytes / 8, sink);
    hipLaunchKernelGGL(write_kernel<uint16_t>, g, b, 0, 0, (uint16_t*)buf, kBytes / 2);
    hipLaunchKernelGGL(write_kernel<uint32_t>, g, b, 0, 0, (uint32_t*)buf, kBytes / 4);
    hipLaunchKernelGGL(write_kernel<uint2>, g, b, 0, 0, (uint2*)buf, kBytes / 8);
    hipLaunchKernelGGL(write_kernel<uint4>, g, b, 0, 0, (uint4*)buf, kBytes / 16);
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    std::printf("{\"bytes_per_stream\": %lld, \"pair_bytes\": %lld}\n", (long long)kBytes,
                (long long)(kBytes / 8 * 12));
    hipFree(buf);
    hipFree(buf2);
    hipFree(sink);
    return 0;
}
