// FETCH_SIZE calibration for the trace kernel's access patterns (diagnostic).
// Each kernel reads every byte of a 512 MiB buffer exactly once (larger than
// the 256 MiB Infinity Cache), so the bytes fetched from HBM are known:
//   stream16 — 16 B per lane, coalesced (the pattern MI355X_MICROARCH.md
//              calibrates: FETCH_SIZE reads 1/2);
//   scalar64 — wave-uniform 64-byte loads (the record streams of the walks);
//   rec48    — one 48-byte record per lane as 3 x 16-byte loads (the light
//              buffer entries' per-lane gathers and LDS staging loads);
//   store4 / store16 — every byte written once, 4 or 16 B per lane (the
//              framebuffer's RGBA8 stores are 4 B per lane).
// Run under rocprofv3 --pmc (FETCH_SIZE, WRITE_SIZE or the TCC_EA0_RDREQ /
// WRREQ size counters) and divide by 512 MiB (tools/calib/rdreq.py).
#include <hip/hip_runtime.h>
#include <cstdio>

constexpr size_t kBytes = 512ull << 20;

__global__ void stream16(const float4* __restrict__ p, size_t n, float* out)
{
    float acc = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x) {
        const float4 v = p[i];
        acc += v.x + v.y + v.z + v.w;
    }
    if (acc == 12345.f) out[0] = acc;
}

// one wave per 64-byte row run: wave w reads rows [w*R, (w+1)*R) uniformly
__global__ void scalar64(const float4* __restrict__ p, size_t rows_per_wave, float* out)
{
    const size_t w = blockIdx.x;  // 64-thread blocks: one wave each
    const float4* q = p + w * rows_per_wave * 4;
    float acc = 0.f;
    for (size_t r = 0; r < rows_per_wave; ++r) {
        const float4 a = q[4 * r], b = q[4 * r + 1], c = q[4 * r + 2], d = q[4 * r + 3];
        acc += (a.x + a.y + a.z + a.w) * (b.x + b.y + b.z + b.w) + (c.x + c.y + c.z + c.w) * (d.x + d.y + d.z + d.w);
    }
    acc += (float)threadIdx.x;
    if (acc == 12345.f) out[0] = acc;
}

__global__ void rec48(const float4* __restrict__ p, size_t nrec, float* out)
{
    float acc = 0.f;
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < nrec; i += (size_t)gridDim.x * blockDim.x) {
        const float4 a = p[3 * i], b = p[3 * i + 1], c = p[3 * i + 2];
        acc += (a.x + a.y + a.z + a.w) * (b.x + b.y + b.z + b.w) + (c.x + c.y + c.z + c.w);
    }
    if (acc == 12345.f) out[0] = acc;
}

// writes: 4 B per lane (the RGBA8 framebuffer's pattern) and 16 B per lane
__global__ void store4(unsigned* __restrict__ p, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = (unsigned)i | 0xFF000000u;
}
__global__ void store16(float4* __restrict__ p, size_t n)
{
    for (size_t i = blockIdx.x * (size_t)blockDim.x + threadIdx.x; i < n; i += (size_t)gridDim.x * blockDim.x)
        p[i] = make_float4((float)i, 1.f, 2.f, 3.f);
}

int main()
{
    float4* p = nullptr;
    float* out = nullptr;
    if (hipMalloc(&p, kBytes) != hipSuccess || hipMalloc(&out, 16) != hipSuccess) return 1;
    hipMemset(p, 0, kBytes);
    hipDeviceSynchronize();
    for (int rep = 0; rep < 3; ++rep) {
        hipLaunchKernelGGL(stream16, dim3(4096), dim3(256), 0, 0, p, kBytes / 16, out);
        const size_t waves = 65536, rows = kBytes / 64 / waves;
        hipLaunchKernelGGL(scalar64, dim3((unsigned)waves), dim3(64), 0, 0, p, rows, out);
        hipLaunchKernelGGL(rec48, dim3(4096), dim3(256), 0, 0, p, kBytes / 48, out);
        hipLaunchKernelGGL(store4, dim3(4096), dim3(256), 0, 0, (unsigned*)p, kBytes / 4);
        hipLaunchKernelGGL(store16, dim3(4096), dim3(256), 0, 0, p, kBytes / 16);
    }
    if (hipDeviceSynchronize() != hipSuccess) return 2;
    std::printf("bytes per launch %zu (rec48 reads %zu)\n", kBytes, kBytes / 48 * 48);
    hipFree(p);
    hipFree(out);
    return 0;
}
