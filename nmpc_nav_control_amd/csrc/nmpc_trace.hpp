// nmpc_trace.hpp -- roctx ranges around the C-ABI entry points (SURVEY.md 5 "Tracing/profiling": the reference
// logs only the wall time of a tick and acados' time_tot, NMPCNavControlROS.cpp:510-513 / :715). With
// `rocprofv3 --marker-trace --kernel-trace` a trace of the ROS-pattern driver separates host packing, copies,
// launches and waits per call; without a tool attached a push / pop is a call into an idle library.
#pragma once

#include <rocprofiler-sdk-roctx/roctx.h>

namespace nmpc {

struct TraceRange {
    explicit TraceRange(const char* name) { roctxRangePushA(name); }
    ~TraceRange() { roctxRangePop(); }
    TraceRange(const TraceRange&) = delete;
    TraceRange& operator=(const TraceRange&) = delete;
};

}  // namespace nmpc
