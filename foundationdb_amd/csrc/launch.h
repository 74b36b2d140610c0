// launch.h — kernel submission for the engine: launch now, or record into a LaunchList.
//
// A LaunchList is one pipeline stage of one batch as data: kernel launches (host stub, grid,
// block, dynamic LDS, argument values) and event records / waits.  The engine records a batch's
// stages on the calling thread and replays them onto their streams from whichever thread submits
// them (the calling thread or the helper), leaving out launches the host knows to be no-ops.
// Every kernel launch of the pipeline goes through fdb_launch.  (Replaying the lists as hipGraphs
// measured slower than direct launches and was removed: DESIGN.md §5.)
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <tuple>
#include <type_traits>
#include <utility>
#include <vector>

namespace fdbcs {

struct LaunchList {
    enum Kind : uint8_t {
        kKernel = 0,
        kTimingRecord = 1,  // event record for phase / roofline timing
        kSyncRecord = 2,    // cross-stream ordering
        kSyncWait = 3,
    };
    struct Rec {
        Kind kind;
        const void* func;
        hipEvent_t event;
        dim3 grid, block;
        uint32_t shmem;
        uint32_t arg0, nargs;  // argument slots [arg0, arg0 + nargs) of argoff / argp
        uint8_t group = 0;     // skip group (t_group when recorded): replay(s, mask) leaves out
                               // kernels whose group is in mask (never a kernel with timing events)
    };
    std::vector<Rec> recs;
    std::vector<uint32_t> argoff;  // byte offset of each argument value in `arena`
    std::vector<unsigned char> arena;
    std::vector<void*> argp;       // finalize(): pointers into arena, in argoff order
    // Per-kernel profile (timing level 3): when set, every recorded kernel is bracketed by two
    // timing events taken from `pool` (created on demand), and (kernel, begin, end) is noted in
    // `spans`; the engine reads the elapsed times once the batch is done.
    struct Profile {
        std::vector<hipEvent_t>* pool;
        size_t* next;
        std::vector<std::pair<const void*, std::pair<hipEvent_t, hipEvent_t>>>* spans;
        hipEvent_t take() {
            if (*next == pool->size()) {
                hipEvent_t e = nullptr;
                if (hipEventCreate(&e) != hipSuccess) return nullptr;
                pool->push_back(e);
            }
            return (*pool)[(*next)++];
        }
    };
    Profile* prof = nullptr;
    // Events around the one kernel `timed_func` (timing level 1, roofline of the dominant kernel),
    // noted in `prof` like the profile spans.
    const void* timed_func = nullptr;

    void clear() {
        recs.clear();
        argoff.clear();
        arena.clear();
        argp.clear();
    }
    template <typename T>
    void push_arg(const T& v) {
        constexpr size_t al = alignof(T) < 16 ? 16 : alignof(T);
        const size_t off = (arena.size() + al - 1) / al * al;
        arena.resize(off + sizeof(T));
        memcpy(arena.data() + off, &v, sizeof(T));
        argoff.push_back((uint32_t)off);
    }
    void finalize() {
        argp.resize(argoff.size());
        for (size_t i = 0; i < argoff.size(); i++) argp[i] = arena.data() + argoff[i];
    }
    // One record, now, on `s` (after finalize()).
    hipError_t issue(const Rec& r, hipStream_t s) {
        switch (r.kind) {
            case kKernel:
                return hipLaunchKernel(r.func, r.grid, r.block, argp.data() + r.arg0, r.shmem, s);
            case kTimingRecord:
            case kSyncRecord:
                return hipEventRecord(r.event, s);
            case kSyncWait:
                return hipStreamWaitEvent(s, r.event, 0);
        }
        return hipSuccess;
    }
    // Direct mode: submit in order (waits and records on `s`), leaving out the kernels of the
    // skip groups in `skip` (whose results the caller knows are not needed).  *skipped counts them.
    hipError_t replay(hipStream_t s, uint8_t skip = 0, int64_t* skipped = nullptr) {
        finalize();
        for (const Rec& r : recs) {
            if (r.kind == kKernel && (r.group & skip)) {
                if (skipped) ++*skipped;
                continue;
            }
            if (hipError_t e = issue(r, s)) return e;
        }
        return hipSuccess;
    }
};

// Non-null while the engine records a stage: fdb_launch / fdb_event append to it.
extern thread_local LaunchList* t_record;
// Skip group of the kernels recorded now (LaunchList::Rec::group).  kGroupEdges: the launches that
// have work only when stage A found candidate intra-batch edges (k_resolve, k_combine,
// k_intra_report); a replay leaves them out once the host has seen that batch's edge count be 0.
constexpr uint8_t kGroupEdges = 1;
extern thread_local uint8_t t_group;
// First failed direct launch since the last take_launch_error().  The engine checks its own
// launches this way rather than with hipGetLastError(), whose per-thread "last error" also holds
// failures of other HIP users in the process (torch shares the runtime) that they never cleared.
extern thread_local hipError_t t_launch_error;
inline hipError_t take_launch_error() {
    const hipError_t e = t_launch_error;
    t_launch_error = hipSuccess;
    return e;
}

template <typename... P, typename... A>
inline void fdb_launch(void (*k)(P...), dim3 grid, dim3 block, uint32_t shmem, hipStream_t s, A&&... a) {
    static_assert(sizeof...(P) == sizeof...(A), "kernel argument count");
    if (LaunchList* L = t_record) {
        LaunchList::Rec r{LaunchList::kKernel, (const void*)k, nullptr, grid, block, shmem, (uint32_t)L->argoff.size(),
                          (uint32_t)sizeof...(P)};
        (L->push_arg(static_cast<std::decay_t<P>>(a)), ...);
        const bool timed = L->prof && (!L->timed_func || L->timed_func == (const void*)k);
        hipEvent_t e0 = timed ? L->prof->take() : nullptr, e1 = timed ? L->prof->take() : nullptr;
        r.group = (e0 && e1) ? 0 : t_group;  // a kernel between timing events is always issued
        if (e0 && e1) L->recs.push_back({LaunchList::kTimingRecord, nullptr, e0, dim3(), dim3(), 0, 0, 0});
        L->recs.push_back(r);
        if (e0 && e1) {
            L->recs.push_back({LaunchList::kTimingRecord, nullptr, e1, dim3(), dim3(), 0, 0, 0});
            L->prof->spans->push_back({(const void*)k, {e0, e1}});
        }
        return;
    }
    std::tuple<std::decay_t<P>...> vals(static_cast<std::decay_t<P>>(a)...);
    std::apply(
        [&](auto&... v) {
            void* args[] = {(void*)&v..., nullptr};
            const hipError_t e = hipLaunchKernel((const void*)k, grid, block, args, shmem, s);
            if (e != hipSuccess && t_launch_error == hipSuccess) t_launch_error = e;
        },
        vals);
}

// kind: LaunchList::kTimingRecord, kSyncRecord or kSyncWait (a wait of `s` on the event).
inline void fdb_event(LaunchList::Kind kind, hipEvent_t e, hipStream_t s) {
    if (!e) return;
    if (LaunchList* L = t_record) {
        L->recs.push_back({kind, nullptr, e, dim3(), dim3(), 0, 0, 0});
        return;
    }
    if (kind == LaunchList::kSyncWait)
        (void)hipStreamWaitEvent(s, e, 0);
    else
        (void)hipEventRecord(e, s);
}

}  // namespace fdbcs
