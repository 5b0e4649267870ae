// plan.hip — launch plans: a training step recorded once and re-issued from C++.
//
// The step is ~300 kernels on two streams (critical path + weight-gradient side stream).  Issued
// from Python, each launch costs ~15 us of host work (tensor views, ctypes argument structs), which
// is more than the GPU needs for most of them: the step ran host-bound (host 4.4 ms vs device
// 4.45 ms critical path, profiles/r01/v10_diag_overlap.log).  ROCm's own graph replay of the same
// capture ran slower on the device (5.5 ms: the two streams' branches lose their concurrency).
//
// A plan is recorded while the caller runs one step: every launch() of the library appends
// (kernel, grid, block, LDS bytes, stream slot, argument bytes), and the caller notes each
// cross-stream ordering edge (alignn_plan_note_wait, after its own event wait).  Replay walks the
// entries: hipLaunchKernel with the stored arguments, hipEventRecord + hipStreamWaitEvent for the
// edges, so the device sees the same kernels, order and stream concurrency as the eager step.
// Stream slot 0 is the stream that was current at alignn_plan_begin; replay puts the caller's
// stream there, every other slot keeps its recorded stream.  Buffers are referenced by address:
// the caller keeps every tensor the step touched alive and in place (trainer.py records inside a
// torch graph capture, whose private memory pool does that, and owns its workspaces), and proves
// it once with alignn_plan_check_ptrs: every device pointer in every recorded argument must lie in
// a range the caller declares it holds for the plan's lifetime.
#include <algorithm>
#include <cstring>
#include <functional>
#include <vector>

#include "common.h"

namespace alignn {

thread_local bool g_recording = false;

struct PlanEntry {
  const void* func;     // kernel (nullptr: stream-ordering edge or timestamp)
  dim3 grid, block;
  uint32_t shmem;
  int slot;             // stream slot (kernel) / waiting stream slot (edge)
  int src;              // edge: slot whose work is waited for
  int event;            // edge: index into Plan::events; timestamp: -1 - index into Plan::stamps
  size_t arg0, nargs;   // kernel: first index into Plan::arg_off, count
  bool reuse;           // edge: the source stream issued nothing since the previous edge from it
                        // (that edge's event is recorded at the same point: wait on it, no new record)
};

struct Plan {
  std::vector<PlanEntry> entries;
  std::vector<unsigned char> args;   // argument bytes (each at its type's alignment, max 16)
  std::vector<size_t> arg_off;
  std::vector<size_t> arg_size;
  std::vector<unsigned char> arg_kind;  // arg_kind<T>() of each argument (common.h)
  std::vector<hipStream_t> streams;  // recorded handles; [0] replaced by the replay stream
  std::vector<hipEvent_t> events;
  std::vector<hipEvent_t> stamps;    // timing events (roofline probes around chosen launches)
  int launches = 0;
};

static thread_local Plan* g_plan = nullptr;

}  // namespace alignn
extern "C" int alignn_plan_destroy(void* plan);
namespace alignn {

static int slot_of(Plan* p, hipStream_t s) {
  for (size_t i = 0; i < p->streams.size(); ++i)
    if (p->streams[i] == s) return (int)i;
  p->streams.push_back(s);
  return (int)p->streams.size() - 1;
}

void record_launch(const void* func, dim3 grid, dim3 block, uint32_t shmem, hipStream_t s, void* const* args,
                   const size_t* sizes, const size_t* aligns, const unsigned char* kinds, int nargs) {
  Plan* p = g_plan;
  if (!p) return;
  PlanEntry e{};
  e.func = func;
  e.grid = grid;
  e.block = block;
  e.shmem = shmem;
  e.slot = slot_of(p, s);
  e.arg0 = p->arg_off.size();
  e.nargs = (size_t)nargs;
  for (int i = 0; i < nargs; ++i) {
    size_t off = p->args.size();
    const size_t al = aligns[i] > 16 ? 16 : aligns[i];
    off = (off + al - 1) / al * al;
    p->args.resize(off + sizes[i]);
    std::memcpy(p->args.data() + off, args[i], sizes[i]);
    p->arg_off.push_back(off);
    p->arg_size.push_back(sizes[i]);
    p->arg_kind.push_back(kinds[i]);
  }
  p->entries.push_back(e);
  p->launches++;
}

__global__ __launch_bounds__(256) void fill_f32_kernel(float* __restrict__ x, int64_t n, float v) {
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n; i += (int64_t)gridDim.x * blockDim.x)
    x[i] = v;
}

// One int64 (the step seed a replayed plan's dropout/jitter kernels read), written by one lane
// through a vector store.
__global__ __launch_bounds__(64) void set_i64_kernel(int64_t* __restrict__ x, int64_t v) {
  if (threadIdx.x == 0) x[0] = v;
}

__global__ __launch_bounds__(256) void copy_f32_kernel(float* __restrict__ dst, const float* __restrict__ src,
                                                       int64_t n) {
  const int64_t n4 = ((reinterpret_cast<uintptr_t>(dst) | reinterpret_cast<uintptr_t>(src)) & 15) ? 0 : n / 4;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x)
    reinterpret_cast<float4*>(dst)[i] = reinterpret_cast<const float4*>(src)[i];
  for (int64_t i = 4 * n4 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    dst[i] = src[i];
}

// x += y elementwise (one add per element: the atom-graph blocks' edge-feature gradient, produced
// on their own stream, folded into the bond-state gradient before the line block's backward)
__global__ __launch_bounds__(256) void add_f32_kernel(float* __restrict__ x, const float* __restrict__ y, int64_t n) {
  const int64_t n4 = ((reinterpret_cast<uintptr_t>(x) | reinterpret_cast<uintptr_t>(y)) & 15) ? 0 : n / 4;
  for (int64_t i = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n4; i += (int64_t)gridDim.x * blockDim.x) {
    float4 a = reinterpret_cast<float4*>(x)[i];
    const float4 b = reinterpret_cast<const float4*>(y)[i];
    a.x += b.x; a.y += b.y; a.z += b.z; a.w += b.w;
    reinterpret_cast<float4*>(x)[i] = a;
  }
  for (int64_t i = 4 * n4 + blockIdx.x * (int64_t)blockDim.x + threadIdx.x; i < n;
       i += (int64_t)gridDim.x * blockDim.x)
    x[i] += y[i];
}

static unsigned blocks_for(int64_t n) { return (unsigned)std::min<int64_t>(std::max<int64_t>(1, (n + 255) / 256), 8192); }

}  // namespace alignn

using namespace alignn;

extern "C" int alignn_plan_begin(void* stream) {
  if (g_plan) {
    set_error("plan_begin: a plan is already being recorded");
    return ALIGNN_E_UNSUPPORTED;
  }
  g_plan = new Plan();
  g_plan->streams.push_back(reinterpret_cast<hipStream_t>(stream));
  g_recording = true;
  return ALIGNN_OK;
}

extern "C" int alignn_plan_note_wait(void* dst_stream, void* src_stream) {
  if (!g_plan) return ALIGNN_OK;
  Plan* p = g_plan;
  PlanEntry e{};
  e.func = nullptr;
  e.slot = slot_of(p, reinterpret_cast<hipStream_t>(dst_stream));
  e.src = slot_of(p, reinterpret_cast<hipStream_t>(src_stream));
  e.event = (int)p->events.size();
  p->events.push_back(nullptr);
  p->entries.push_back(e);
  return ALIGNN_OK;
}

// Timestamp entry on `stream` (replay records a timing event there); returns its index, or -1
// when no plan is being recorded.
extern "C" int alignn_plan_note_timestamp(void* stream) {
  if (!g_plan) return -1;
  Plan* p = g_plan;
  PlanEntry e{};
  e.func = nullptr;
  e.slot = slot_of(p, reinterpret_cast<hipStream_t>(stream));
  const int idx = (int)p->stamps.size();
  e.event = -1 - idx;
  p->stamps.push_back(nullptr);
  p->entries.push_back(e);
  return idx;
}

extern "C" void* alignn_plan_end(void) {
  Plan* p = g_plan;
  g_plan = nullptr;
  g_recording = false;
  if (!p) {
    set_error("plan_end: no plan is being recorded");
    return nullptr;
  }
  // an edge from a stream that issued nothing since its previous edge (two streams waiting on one
  // point, e.g. the aux and side streams both after a gate kernel of the main stream) reuses that
  // edge's event: one marker on the source stream instead of two
  {
    std::vector<int> last_edge(p->streams.size(), -1);   // per source slot: event of its latest edge
    for (PlanEntry& e : p->entries) {
      if (e.func || e.event < 0) {   // the slot issued work (or a timestamp)
        last_edge[(size_t)e.slot] = -1;
        continue;
      }
      const int prev = last_edge[(size_t)e.src];
      if (prev >= 0) {
        e.reuse = true;
        e.event = prev;
      } else {
        last_edge[(size_t)e.src] = e.event;
      }
      last_edge[(size_t)e.slot] = -1;   // the waiting stream's later work now also follows the source
    }
  }
  bool ok = true;
  // Cross-stream edges inside the step: no system-scope fence at the record.  The producing kernel's
  // end-of-kernel release (agent scope: the XCD L2s written back, gfx950 memory model) already makes its
  // writes visible to every kernel of the device, as it does for the next kernel of its own stream; the
  // default event adds a system-scope writeback that holds the source stream ~4 us per edge
  // (tools/probe/marker_cost.hip: 7.2 us per kernel pair -> 11.1 with a default event between them, 8.8
  // without the system fence).  The last edge from each other slot into slot 0 — the joins after which
  // the caller's stream, torch ops and device-to-host copies (loss.item()) read the step's results —
  // keeps the default, system-scope event: visibility beyond the device's kernels is then not assumed.
  std::vector<char> fenced(p->events.size(), 0);
  {
    std::vector<int> last_join(p->streams.size(), -1);   // per source slot: its last edge into slot 0
    for (const PlanEntry& e : p->entries)
      if (!e.func && e.event >= 0 && e.slot == 0) last_join[(size_t)e.src] = e.event;
    for (int ev : last_join)
      if (ev >= 0) fenced[(size_t)ev] = 1;
  }
  for (size_t i = 0; i < p->events.size(); ++i)
    ok = ok && hipEventCreateWithFlags(&p->events[i], fenced[i] ? hipEventDisableTiming
                                                                 : (hipEventDisableTiming | hipEventDisableSystemFence))
                   == hipSuccess;
  for (auto& ev : p->stamps) ok = ok && hipEventCreate(&ev) == hipSuccess;
  if (!ok) {
    set_error("plan_end: event creation failed");
    alignn_plan_destroy(p);
    return nullptr;
  }
  return p;
}

extern "C" int alignn_plan_abort(void) {
  delete g_plan;
  g_plan = nullptr;
  g_recording = false;
  return ALIGNN_OK;
}

extern "C" int alignn_plan_info(const void* plan, int64_t* launches, int64_t* waits, int64_t* streams,
                                int64_t* arg_bytes) {
  const Plan* p = reinterpret_cast<const Plan*>(plan);
  if (!p) return ALIGNN_E_BAD_SHAPE;
  if (launches) *launches = p->launches;
  if (waits) *waits = (int64_t)p->events.size();
  if (streams) *streams = (int64_t)p->streams.size();
  if (arg_bytes) *arg_bytes = (int64_t)p->args.size();
  return ALIGNN_OK;
}

// Introspection (tools/plan_dump.py): entry i as (kind, slot, src) — kind 0 kernel, 1 stream edge
// (slot waits for src), 2 timestamp — and, for kernels, the device function's name.  Returns the
// entry count; fills at most `cap` entries.
extern "C" int64_t alignn_plan_entries(const void* plan, int32_t* kind_slot_src, const char** names, int64_t cap) {
  const Plan* p = reinterpret_cast<const Plan*>(plan);
  if (!p) return -1;
  const int64_t n = (int64_t)p->entries.size();
  for (int64_t i = 0; i < n && i < cap; ++i) {
    const PlanEntry& e = p->entries[(size_t)i];
    kind_slot_src[3 * i] = e.func ? 0 : (e.event < 0 ? 2 : 1);
    kind_slot_src[3 * i + 1] = e.slot;
    kind_slot_src[3 * i + 2] = e.func ? -1 : e.src;
    if (names) names[i] = e.func ? hipKernelNameRefByPtr(e.func, p->streams[(size_t)e.slot]) : nullptr;
  }
  return n;
}

extern "C" int alignn_plan_replay(void* plan, void* stream) {
  Plan* p = reinterpret_cast<Plan*>(plan);
  if (!p) return ALIGNN_E_BAD_SHAPE;
  if (g_recording) {
    set_error("plan_replay: not allowed while a plan is being recorded");
    return ALIGNN_E_UNSUPPORTED;
  }
  p->streams[0] = reinterpret_cast<hipStream_t>(stream);
  std::vector<void*> ptrs;
  for (const PlanEntry& e : p->entries) {
    if (e.func) {
      ptrs.resize(e.nargs + 1);
      for (size_t i = 0; i < e.nargs; ++i) ptrs[i] = p->args.data() + p->arg_off[e.arg0 + i];
      hipError_t r = hipLaunchKernel(e.func, e.grid, e.block, ptrs.data(), e.shmem, p->streams[e.slot]);
      if (r != hipSuccess) return hip_status(r, "plan_replay: hipLaunchKernel");
    } else if (e.event < 0) {
      hipError_t r = hipEventRecord(p->stamps[-1 - e.event], p->streams[e.slot]);
      if (r != hipSuccess) return hip_status(r, "plan_replay: timestamp");
    } else {
      hipError_t r = e.reuse ? hipSuccess : hipEventRecord(p->events[e.event], p->streams[e.src]);
      if (r == hipSuccess) r = hipStreamWaitEvent(p->streams[e.slot], p->events[e.event], 0);
      if (r != hipSuccess) return hip_status(r, "plan_replay: stream edge");
    }
  }
  return ALIGNN_OK;
}

// Serialised replay (roofline probes): every launch and timestamp in recorded issue order on
// `stream` alone, the cross-stream edges dropped — issue order already satisfies them (a wait is
// noted after the work it waits for was issued).  The timestamps then bracket each kernel alone on
// the device, as a counter-collection pass runs it, instead of including the time it queued behind
// the other streams' kernels.
extern "C" int alignn_plan_replay_serial(void* plan, void* stream) {
  Plan* p = reinterpret_cast<Plan*>(plan);
  if (!p) return ALIGNN_E_BAD_SHAPE;
  if (g_recording) {
    set_error("plan_replay_serial: not allowed while a plan is being recorded");
    return ALIGNN_E_UNSUPPORTED;
  }
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  std::vector<void*> ptrs;
  for (const PlanEntry& e : p->entries) {
    if (e.func) {
      ptrs.resize(e.nargs + 1);
      for (size_t i = 0; i < e.nargs; ++i) ptrs[i] = p->args.data() + p->arg_off[e.arg0 + i];
      hipError_t r = hipLaunchKernel(e.func, e.grid, e.block, ptrs.data(), e.shmem, s);
      if (r != hipSuccess) return hip_status(r, "plan_replay_serial: hipLaunchKernel");
    } else if (e.event < 0) {
      hipError_t r = hipEventRecord(p->stamps[-1 - e.event], s);
      if (r != hipSuccess) return hip_status(r, "plan_replay_serial: timestamp");
    }
  }
  return ALIGNN_OK;
}

extern "C" int alignn_plan_destroy(void* plan) {
  Plan* p = reinterpret_cast<Plan*>(plan);
  if (!p) return ALIGNN_OK;
  for (auto& ev : p->events)
    if (ev) (void)hipEventDestroy(ev);
  for (auto& ev : p->stamps)
    if (ev) (void)hipEventDestroy(ev);
  delete p;
  return ALIGNN_OK;
}

// Ownership check of a recorded plan.  ranges: n pairs [lo, hi) of device byte addresses the caller
// holds for the plan's lifetime.  Every non-null pointer argument, and every 8-byte word of a
// struct argument that the HIP runtime resolves to device memory, must fall in one of them;
// otherwise the first offending value and its launch index are returned with ALIGNN_E_BAD_SHAPE.
extern "C" int alignn_plan_check_ptrs(const void* plan, const uint64_t* ranges, int64_t n, uint64_t* bad_value,
                                      int64_t* bad_launch, int64_t* checked) {
  const Plan* p = reinterpret_cast<const Plan*>(plan);
  if (!p || n < 0 || (n > 0 && !ranges)) return ALIGNN_E_BAD_SHAPE;
  std::vector<std::pair<uint64_t, uint64_t>> rs;
  for (int64_t i = 0; i < n; ++i) rs.emplace_back(ranges[2 * i], ranges[2 * i + 1]);
  auto held = [&](uint64_t v) {  // ranges may nest or overlap (views inside pool segments)
    for (const auto& r : rs)
      if (v >= r.first && v < r.second) return true;
    return false;
  };
  auto device_word = [](uint64_t v) {
    if (v < (1ull << 32) || v >= (1ull << 47)) return false;  // not a user-space device address
    hipPointerAttribute_t at;
    const hipError_t r = hipPointerGetAttributes(&at, reinterpret_cast<const void*>(v));
    (void)hipGetLastError();  // an unknown address is an ordinary answer here, not a pending error
    return r == hipSuccess && at.type == hipMemoryTypeDevice;
  };
  int64_t launch_idx = -1, nchecked = 0;
  for (const PlanEntry& e : p->entries) {
    if (!e.func) continue;
    ++launch_idx;
    for (size_t a = 0; a < e.nargs; ++a) {
      const size_t j = e.arg0 + a;
      const unsigned char* b = p->args.data() + p->arg_off[j];
      if (p->arg_kind[j] == 1) {
        uint64_t v;
        std::memcpy(&v, b, sizeof v);
        if (!v) continue;
        ++nchecked;
        if (!held(v)) {
          if (bad_value) *bad_value = v;
          if (bad_launch) *bad_launch = launch_idx;
          set_error("plan_check_ptrs: launch %lld argument %zu points at 0x%llx, outside every held buffer",
                    (long long)launch_idx, a, (unsigned long long)v);
          return ALIGNN_E_BAD_SHAPE;
        }
      } else if (p->arg_kind[j] == 2) {
        for (size_t o = 0; o + 8 <= p->arg_size[j]; o += 8) {
          uint64_t v;
          std::memcpy(&v, b + o, sizeof v);
          if (!v || held(v)) { nchecked += v ? 1 : 0; continue; }
          if (device_word(v)) {
            if (bad_value) *bad_value = v;
            if (bad_launch) *bad_launch = launch_idx;
            set_error("plan_check_ptrs: launch %lld argument %zu (struct word %zu) points at 0x%llx, outside "
                      "every held buffer", (long long)launch_idx, a, o / 8, (unsigned long long)v);
            return ALIGNN_E_BAD_SHAPE;
          }
        }
      }
    }
  }
  if (checked) *checked = nchecked;
  return ALIGNN_OK;
}

// Which of n caller ranges [lo, hi) the recorded plan reads or writes through any pointer argument
// or struct-argument word: hit[i] = 1 if some such value lies in range i (a struct word that only
// looks like an address marks a range too — harmless, the caller then copies one buffer more).
// trainer._rebind copies a new batch only into the captured batch's buffers a plan touches.
extern "C" int alignn_plan_refs(const void* plan, const uint64_t* ranges, int64_t n, int32_t* hit) {
  const Plan* p = reinterpret_cast<const Plan*>(plan);
  if (!p || n < 0 || (n > 0 && (!ranges || !hit))) return ALIGNN_E_BAD_SHAPE;
  auto mark = [&](uint64_t v) {
    if (!v) return;
    for (int64_t i = 0; i < n; ++i)
      if (v >= ranges[2 * i] && v < ranges[2 * i + 1]) hit[i] = 1;
  };
  for (int64_t i = 0; i < n; ++i) hit[i] = 0;
  for (const PlanEntry& e : p->entries) {
    if (!e.func) continue;
    for (size_t a = 0; a < e.nargs; ++a) {
      const size_t j = e.arg0 + a;
      const unsigned char* b = p->args.data() + p->arg_off[j];
      if (p->arg_kind[j] == 1) {
        uint64_t v;
        std::memcpy(&v, b, sizeof v);
        mark(v);
      } else if (p->arg_kind[j] == 2) {
        for (size_t o = 0; o + 8 <= p->arg_size[j]; o += 8) {
          uint64_t v;
          std::memcpy(&v, b + o, sizeof v);
          mark(v);
        }
      }
    }
  }
  return ALIGNN_OK;
}

// Device time between two timestamps of the last replay (call after it has completed).
extern "C" int alignn_plan_elapsed_ms(void* plan, int32_t i0, int32_t i1, float* ms) {
  Plan* p = reinterpret_cast<Plan*>(plan);
  if (!p || i0 < 0 || i1 < 0 || i0 >= (int)p->stamps.size() || i1 >= (int)p->stamps.size() || !ms)
    return ALIGNN_E_BAD_SHAPE;
  hipError_t r = hipEventElapsedTime(ms, p->stamps[i0], p->stamps[i1]);
  if (r != hipSuccess) return hip_status(r, "plan_elapsed_ms");
  return ALIGNN_OK;
}

// Node census of a captured HIP graph: kernel nodes and everything else (memcpy, memset, host,
// child graphs ...; event and empty nodes are not counted).  A plan recorded during that capture
// is complete when its launch count equals the kernel count and `other` is 0.
extern "C" int alignn_graph_census(void* graph, int64_t* kernels, int64_t* other) {
  hipGraph_t g = reinterpret_cast<hipGraph_t>(graph);
  size_t n = 0;
  hipError_t r = hipGraphGetNodes(g, nullptr, &n);
  if (r != hipSuccess) return hip_status(r, "graph_census: hipGraphGetNodes");
  std::vector<hipGraphNode_t> nodes(n);
  if (n) {
    r = hipGraphGetNodes(g, nodes.data(), &n);
    if (r != hipSuccess) return hip_status(r, "graph_census: hipGraphGetNodes");
  }
  int64_t k = 0, o = 0;
  for (size_t i = 0; i < n; ++i) {
    hipGraphNodeType t;
    r = hipGraphNodeGetType(nodes[i], &t);
    if (r != hipSuccess) return hip_status(r, "graph_census: hipGraphNodeGetType");
    if (t == hipGraphNodeTypeKernel) ++k;
    else if (t != hipGraphNodeTypeEmpty && t != hipGraphNodeTypeWaitEvent && t != hipGraphNodeTypeEventRecord) ++o;
  }
  *kernels = k;
  *other = o;
  return ALIGNN_OK;
}

// Dependency check of a recorded plan against the HIP graph captured while it was recorded.  The
// plan orders work by its per-slot program order and the cross-stream edges noted with
// alignn_plan_note_wait; the captured graph by the dependencies the stream capture derived from
// every event wait — including waits issued without noting them (a torch-level wait_stream), which
// a replayed plan silently drops (round 3: an un-noted join let the next phase overwrite buffers the
// side stream still read).  Checks, with the kernel nodes matched to the recorded launches in
// creation order (same kernel function, grid and block required):
//   1. every graph dependency between two kernels (directly or through empty / event nodes) is a
//      happens-before of the plan (vector clocks over the slots);
//   2. the plan ends joined: every slot's last kernel happens before the end of slot 0 (a stream
//      capture must end with every forked stream joined; the next phase starts on slot 0 alone).
// On failure: ALIGNN_E_BAD_SHAPE, *bad_from / *bad_to = the launch indices of the first edge the
// plan lacks (bad_to = -1: an unjoined slot, bad_from = its last launch).
extern "C" int alignn_plan_check_deps(const void* plan, void* graph, int64_t* bad_from, int64_t* bad_to,
                                      int64_t* graph_edges) {
  const Plan* p = reinterpret_cast<const Plan*>(plan);
  hipGraph_t g = reinterpret_cast<hipGraph_t>(graph);
  if (!p || !g) return ALIGNN_E_BAD_SHAPE;
  if (bad_from) *bad_from = -1;
  if (bad_to) *bad_to = -1;
  // plan happens-before: vector clocks over the stream slots
  const size_t S = p->streams.size();
  std::vector<std::vector<int64_t>> clk(S, std::vector<int64_t>(S, 0));
  std::vector<std::vector<int64_t>> vc;      // per launch: clock of its slot when it was issued
  std::vector<int> lslot;
  std::vector<int64_t> lseq;
  std::vector<const void*> lfunc;
  std::vector<dim3> lgrid, lblock;
  for (const PlanEntry& e : p->entries) {
    if (e.func) {
      clk[e.slot][e.slot] += 1;
      vc.push_back(clk[e.slot]);
      lslot.push_back(e.slot);
      lseq.push_back(clk[e.slot][e.slot]);
      lfunc.push_back(e.func);
      lgrid.push_back(e.grid);
      lblock.push_back(e.block);
    } else if (e.event >= 0) {
      for (size_t k = 0; k < S; ++k) clk[e.slot][k] = std::max(clk[e.slot][k], clk[e.src][k]);
    }
  }
  auto hb = [&](int64_t a, int64_t b) { return vc[b][lslot[a]] >= lseq[a]; };
  // graph nodes, kernel nodes in creation order
  size_t n = 0;
  hipError_t r = hipGraphGetNodes(g, nullptr, &n);
  if (r != hipSuccess) return hip_status(r, "plan_check_deps: hipGraphGetNodes");
  std::vector<hipGraphNode_t> nodes(n);
  if (n) {
    r = hipGraphGetNodes(g, nodes.data(), &n);
    if (r != hipSuccess) return hip_status(r, "plan_check_deps: hipGraphGetNodes");
  }
  // kernel nodes -> recorded launches: the same kernel, grid and block and the same argument bytes
  // (the node's kernelParams); among identical launches, in order.  hipGraphGetNodes does not list
  // the nodes of a multi-stream capture in issue order.
  std::vector<int64_t> launch_of;   // node index -> launch index (-1: not a kernel)
  std::vector<std::pair<hipGraphNode_t, int64_t>> index;
  std::vector<char> taken(lfunc.size(), 0);
  std::vector<size_t> lentry;       // launch index -> entry index (argument bytes)
  for (size_t i = 0; i < p->entries.size(); ++i)
    if (p->entries[i].func) lentry.push_back(i);
  int64_t k = 0;
  for (size_t i = 0; i < n; ++i) {
    hipGraphNodeType t;
    r = hipGraphNodeGetType(nodes[i], &t);
    if (r != hipSuccess) return hip_status(r, "plan_check_deps: hipGraphNodeGetType");
    index.emplace_back(nodes[i], (int64_t)i);
    if (t != hipGraphNodeTypeKernel) {
      launch_of.push_back(-1);
      continue;
    }
    hipKernelNodeParams kp{};
    r = hipGraphKernelNodeGetParams(nodes[i], &kp);
    if (r != hipSuccess) return hip_status(r, "plan_check_deps: hipGraphKernelNodeGetParams");
    int64_t hit = -1;
    for (size_t a = 0; a < lfunc.size() && hit < 0; ++a) {
      if (taken[a] || kp.func != lfunc[a] || kp.gridDim.x != lgrid[a].x || kp.gridDim.y != lgrid[a].y ||
          kp.gridDim.z != lgrid[a].z || kp.blockDim.x != lblock[a].x || kp.blockDim.y != lblock[a].y ||
          kp.blockDim.z != lblock[a].z)
        continue;
      const PlanEntry& e = p->entries[lentry[a]];
      bool same = true;
      if (kp.kernelParams) {
        for (size_t j = 0; j < e.nargs && same; ++j) {
          const size_t q = e.arg0 + j;
          same = kp.kernelParams[j] && std::memcmp(kp.kernelParams[j], p->args.data() + p->arg_off[q], p->arg_size[q]) == 0;
        }
      }
      if (same) hit = (int64_t)a;
    }
    if (hit < 0) {
      set_error("plan_check_deps: kernel node %zu (func %p) matches no launch of the plan", i, kp.func);
      return ALIGNN_E_BAD_SHAPE;
    }
    taken[hit] = 1;
    launch_of.push_back(hit);
    ++k;
  }
  if (k != (int64_t)lfunc.size()) {
    set_error("plan_check_deps: the graph holds %lld kernel nodes, the plan %zu launches", (long long)k, lfunc.size());
    return ALIGNN_E_BAD_SHAPE;
  }
  std::sort(index.begin(), index.end());
  auto node_idx = [&](hipGraphNode_t h) -> int64_t {
    auto it = std::lower_bound(index.begin(), index.end(), std::make_pair(h, (int64_t)-1));
    return (it != index.end() && it->first == h) ? it->second : -1;
  };
  // nearest kernel ancestors through non-kernel nodes (memoised per node)
  std::vector<std::vector<int64_t>> kanc(n);
  std::vector<char> done(n, 0);
  std::vector<hipGraphNode_t> deps;
  auto direct = [&](size_t i, std::vector<int64_t>& out) -> int {
    size_t nd = 0;
    hipError_t rr = hipGraphNodeGetDependencies(nodes[i], nullptr, &nd);
    if (rr != hipSuccess) return hip_status(rr, "plan_check_deps: hipGraphNodeGetDependencies");
    deps.resize(nd);
    if (nd) {
      rr = hipGraphNodeGetDependencies(nodes[i], deps.data(), &nd);
      if (rr != hipSuccess) return hip_status(rr, "plan_check_deps: hipGraphNodeGetDependencies");
    }
    for (size_t j = 0; j < nd; ++j) {
      const int64_t d = node_idx(deps[j]);
      if (d < 0) {
        set_error("plan_check_deps: a dependency outside the graph's node list");
        return ALIGNN_E_BAD_SHAPE;
      }
      out.push_back(d);
    }
    return ALIGNN_OK;
  };
  // kernel ancestors of node i: iterative DFS over non-kernel predecessors
  std::function<int(size_t)> resolve = [&](size_t i) -> int {
    if (done[i]) return ALIGNN_OK;
    std::vector<int64_t> ds;
    int rc = direct(i, ds);
    if (rc) return rc;
    std::vector<int64_t> acc;
    for (int64_t d : ds) {
      if (launch_of[d] >= 0) {
        acc.push_back(launch_of[d]);
      } else {
        rc = resolve((size_t)d);
        if (rc) return rc;
        acc.insert(acc.end(), kanc[d].begin(), kanc[d].end());
      }
    }
    std::sort(acc.begin(), acc.end());
    acc.erase(std::unique(acc.begin(), acc.end()), acc.end());
    kanc[i] = std::move(acc);
    done[i] = 1;
    return ALIGNN_OK;
  };
  int64_t edges = 0;
  for (size_t i = 0; i < n; ++i) {
    if (launch_of[i] < 0) continue;
    int rc = resolve(i);
    if (rc) return rc;
    for (int64_t a : kanc[i]) {
      ++edges;
      if (!hb(a, launch_of[i])) {
        if (bad_from) *bad_from = a;
        if (bad_to) *bad_to = launch_of[i];
        set_error("plan_check_deps: the captured graph orders launch %lld (slot %d) before launch %lld (slot %d), "
                  "the plan does not (a cross-stream wait that was not noted)", (long long)a, lslot[a],
                  (long long)launch_of[i], lslot[launch_of[i]]);
        return ALIGNN_E_BAD_SHAPE;
      }
    }
  }
  if (graph_edges) *graph_edges = edges;
  // ends joined: slot 0's final clock covers every slot's last launch
  for (size_t s = 1; s < S; ++s) {
    if (clk[0][s] < clk[s][s]) {
      int64_t last = -1;
      for (size_t a = 0; a < lslot.size(); ++a)
        if (lslot[a] == (int)s) last = (int64_t)a;
      if (bad_from) *bad_from = last;
      set_error("plan_check_deps: stream slot %zu's last launch (%lld) is not joined into slot 0 at the end of the "
                "plan (the next phase could overtake it)", s, (long long)last);
      return ALIGNN_E_BAD_SHAPE;
    }
  }
  return ALIGNN_OK;
}

extern "C" int alignn_fill_f32(float* x, int64_t n, float value, void* stream) {
  if (n < 0) return ALIGNN_E_BAD_SHAPE;
  if (n == 0) return ALIGNN_OK;
  launch(fill_f32_kernel, dim3(blocks_for(n)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), x, n, value);
  ALIGNN_LAUNCH_CHECK("fill_f32_kernel");
  return ALIGNN_OK;
}

extern "C" int alignn_set_i64(int64_t* x, int64_t value, void* stream) {
  if (!x) return ALIGNN_E_BAD_SHAPE;
  launch(set_i64_kernel, dim3(1), dim3(64), 0, reinterpret_cast<hipStream_t>(stream), x, value);
  ALIGNN_LAUNCH_CHECK("set_i64_kernel");
  return ALIGNN_OK;
}

extern "C" int alignn_copy_f32(float* dst, const float* src, int64_t n, void* stream) {
  if (n < 0) return ALIGNN_E_BAD_SHAPE;
  if (n == 0) return ALIGNN_OK;
  launch(copy_f32_kernel, dim3(blocks_for((n + 3) / 4)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), dst,
         src, n);
  ALIGNN_LAUNCH_CHECK("copy_f32_kernel");
  return ALIGNN_OK;
}

extern "C" int alignn_add_f32(float* x, const float* y, int64_t n, void* stream) {
  if (n < 0) return ALIGNN_E_BAD_SHAPE;
  if (n == 0) return ALIGNN_OK;
  launch(add_f32_kernel, dim3(blocks_for((n + 3) / 4)), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), x, y, n);
  ALIGNN_LAUNCH_CHECK("add_f32_kernel");
  return ALIGNN_OK;
}

// A HIP stream of the library's own (non-blocking, given priority): an execution context's side / aux
// streams must be distinct from every stream torch hands out from its pool, since the context tells
// its stream roles apart by handle.
extern "C" int alignn_stream_create(int32_t priority, void** out) {
  if (!out) return ALIGNN_E_BAD_SHAPE;
  hipStream_t s = nullptr;
  hipError_t e = hipStreamCreateWithPriority(&s, hipStreamNonBlocking, (int)priority);
  if (e != hipSuccess) {
    set_error("hipStreamCreateWithPriority: %s", hipGetErrorString(e));
    return ALIGNN_E_HIP;
  }
  *out = reinterpret_cast<void*>(s);
  return ALIGNN_OK;
}

// A stream on a hardware queue of its own: a CU-masked stream (every CU enabled) is given a new queue
// instead of one from the process's pool of GPU_MAX_HW_QUEUES (4 here), so a batch-preparation stream
// cannot end up sharing a queue — and its in-order dispatch — with one of the step's streams.
extern "C" int alignn_stream_create_dedicated(void** out) {
  if (!out) return ALIGNN_E_BAD_SHAPE;
  int dev = 0, cus = 0;
  hipError_t e = hipGetDevice(&dev);
  if (e == hipSuccess) e = hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
  if (e != hipSuccess || cus <= 0) {
    set_error("alignn_stream_create_dedicated: CU count: %s", hipGetErrorString(e));
    return ALIGNN_E_HIP;
  }
  std::vector<uint32_t> mask((size_t)(cus + 31) / 32, 0xffffffffu);
  if (cus % 32) mask.back() = (1u << (cus % 32)) - 1u;
  hipStream_t s = nullptr;
  e = hipExtStreamCreateWithCUMask(&s, (uint32_t)mask.size(), mask.data());
  if (e != hipSuccess) {
    set_error("hipExtStreamCreateWithCUMask: %s", hipGetErrorString(e));
    return ALIGNN_E_HIP;
  }
  *out = reinterpret_cast<void*>(s);
  return ALIGNN_OK;
}

extern "C" int alignn_stream_destroy(void* stream) {
  if (!stream) return ALIGNN_OK;
  hipStream_t s = reinterpret_cast<hipStream_t>(stream);
  hipError_t e = hipStreamSynchronize(s);
  if (e == hipSuccess) e = hipStreamDestroy(s);
  if (e != hipSuccess) {
    set_error("hipStreamDestroy: %s", hipGetErrorString(e));
    return ALIGNN_E_HIP;
  }
  return ALIGNN_OK;
}
