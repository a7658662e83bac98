// nmpc_trace.hpp -- roctx ranges around the C-ABI entry points (SURVEY.md 5 "Tracing/profiling": the reference
// logs only the wall time of a tick and acados' time_tot, NMPCNavControlROS.cpp:510-513 / :715). With
// `rocprofv3 --marker-trace --kernel-trace` a trace of the ROS-pattern driver separates host packing, copies,
// launches and waits per call; without a tool attached a push / pop is a call into an idle library.
#pragma once

// Built with NMPC_ROCTX (the Makefile sets it when rocprofiler-sdk's roctx is installed); otherwise a no-op.
#ifdef NMPC_ROCTX
#include <rocprofiler-sdk-roctx/roctx.h>
#endif

namespace nmpc {

struct TraceRange {
#ifdef NMPC_ROCTX
    explicit TraceRange(const char* name) { roctxRangePushA(name); }
    ~TraceRange() { roctxRangePop(); }
#else
    explicit TraceRange(const char*) {}
#endif
    TraceRange(const TraceRange&) = delete;
    TraceRange& operator=(const TraceRange&) = delete;
};

}  // namespace nmpc
