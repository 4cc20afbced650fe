// launch_cost.hip — host cost of the calls around one forward launch (sphrt_forward_f32:
// hipStreamGetDevice + hipGetDevice in StreamGuard, hipLaunchKernelGGL with the forward's 21
// arguments, hipGetLastError), each on its own, against an idle and a busy queue.
//
//   hipcc --offload-arch=gfx950 -O2 tools/launch_cost.hip -o gpurun_out/launch_cost
#include <hip/hip_runtime.h>

#include <chrono>
#include <cstdint>
#include <cstdio>

struct Big {   // the forward's by-value arguments, about the same size (21 values)
    const void* p[12];
    int64_t v[8];
    int c;
};

__global__ void k_args(const void* a0, const void* a1, const void* a2, const void* a3,
                       const void* a4, const void* a5, const void* a6, const void* a7,
                       int64_t n0, int64_t n1, int64_t n2, float* out, int64_t n3, int64_t n4,
                       int64_t n5, int64_t n6, int64_t n7, int c0, int c1, int c2,
                       const void* a8) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && n0 == -12345) out[0] = (float)(n1 + c0);
}

__global__ void k_struct(Big b, float* out) {
    if (threadIdx.x == 0 && blockIdx.x == 0 && b.v[0] == -12345) out[0] = (float)b.c;
}

template <typename F>
static double per_call_us(F f, int reps, hipStream_t st) {
    hipStreamSynchronize(st);
    for (int i = 0; i < 20; ++i) f();
    hipStreamSynchronize(st);
    auto t0 = std::chrono::steady_clock::now();
    for (int i = 0; i < reps; ++i) f();
    auto t1 = std::chrono::steady_clock::now();
    hipStreamSynchronize(st);
    return std::chrono::duration<double, std::micro>(t1 - t0).count() / reps;
}

int main() {
    hipStream_t st;
    hipStreamCreateWithFlags(&st, hipStreamNonBlocking);
    float* out;
    hipMalloc(&out, 4);
    const int reps = 400;
    const dim3 grid(1473), block(224);
    Big b{};
    auto launch_args = [&] {
        hipLaunchKernelGGL(k_args, grid, block, 4096, st, out, out, out, out, out, out, out, out,
                           (int64_t)1, (int64_t)2, (int64_t)3, out, (int64_t)4, (int64_t)5,
                           (int64_t)6, (int64_t)7, (int64_t)8, 1, 2, 3, (const void*)out);
    };
    auto launch_struct = [&] { hipLaunchKernelGGL(k_struct, grid, block, 4096, st, b, out); };
    int dev;
    hipDevice_t d;
    printf("{\"hipGetDevice_us\": %.3f, ", per_call_us([&] { hipGetDevice(&dev); }, 20000, st));
    printf("\"hipStreamGetDevice_us\": %.3f, ",
           per_call_us([&] { hipStreamGetDevice(st, &d); }, 20000, st));
    printf("\"hipGetLastError_us\": %.3f, ", per_call_us([&] { (void)hipGetLastError(); }, 20000, st));
    printf("\"launch_21_args_us\": %.3f, ", per_call_us(launch_args, reps, st));
    printf("\"launch_struct_us\": %.3f, ", per_call_us(launch_struct, reps, st));
    printf("\"launch_plus_guards_us\": %.3f}\n", per_call_us([&] {
        hipStreamGetDevice(st, &d);
        hipGetDevice(&dev);
        launch_args();
        (void)hipGetLastError();
    }, reps, st));
    return 0;
}
