// rt_cpu.hpp — internal interface of the CPU backend (rt_cpu.cpp) to the C
// ABI in rt_kernels.hip.  Host code only.
#ifndef RT_AMD_RT_CPU_HPP
#define RT_AMD_RT_CPU_HPP

#include "../../include/rt.h"

namespace rt {
// (Re)build the host scene from the flat post-Pretraitement scene.
int cpu_upload(void** handle, const rt_scene_flat* s);
void cpu_free(void* handle);
// Render `rows` output rows of frame f (slab or band set) on `threads` host
// threads (<= 0: all); either output may be null.  *ms = wall time.
int cpu_render(const void* handle, int threads, const rt_frame* f, int rows, uint8_t* rgba8, float* rgb, double* ms);
}  // namespace rt

#endif  // RT_AMD_RT_CPU_HPP
