// prof.h — internal (not exported): the per-launch profiling spans of gw_profile, shared by the
// library's translation units.  gridenv.hip owns the env's timing events; a span opened here
// hands them to the next launches made through gwprof::launch on this thread (start = the first
// launch's begin, stop = every launch's end, the last one wins: hipExtLaunchKernelGGL carries
// them in the dispatch itself, no marker packets between the kernels).  The span kinds are the
// GW_SPAN_* values of include/gridenv.h.
#pragma once
#include <hip/hip_runtime.h>
#include <hip/hip_ext.h>

#include <cstddef>
#include <cstdint>

#include "gridenv.h"

namespace gwprof {

// events handed to the next launch(es) on this thread; t_bind_stop: a pipeline event bound to a
// launch the same way when no span is open (gridenv.hip: obs_done, world_ev)
extern thread_local hipEvent_t t_span_start, t_span_stop, t_bind_stop;

// open a span of `env` if it is profiling (returns false otherwise: nothing to close)
bool span_begin(void *env, size_t *idx);
// close it: record (kind, start, stop) if a kernel was launched in it
void span_end(void *env, size_t idx, int kind);

template <typename F, typename... Args>
inline void launch(F kernel, dim3 grid, dim3 block, size_t lds, hipStream_t s, Args... args) {
    hipEvent_t stop = t_span_stop ? t_span_stop : t_bind_stop;
    if (stop) {
        hipExtLaunchKernelGGL(kernel, grid, block, (uint32_t)lds, s, t_span_start, stop, 0u, args...);
        t_span_start = nullptr;
    } else {
        hipLaunchKernelGGL(kernel, grid, block, lds, s, args...);
    }
}

// RAII span for the ops that take an env handle (actor_ops.hip, gw_obs_patch): every launch in
// scope made through gwprof::launch belongs to one span of `kind`
struct Span {
    void *env;
    size_t idx = 0;
    bool open;
    int kind;
    Span(void *e, int k) : env(e), open(e && span_begin(e, &idx)), kind(k) {}
    ~Span() {
        if (open) span_end(env, idx, kind);
    }
    Span(const Span &) = delete;
    Span &operator=(const Span &) = delete;
};

}  // namespace gwprof
