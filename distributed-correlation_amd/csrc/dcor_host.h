// dcor_host.h -- host-side internals shared by the C-ABI translation units (dcor_capi.cpp,
// dcor_grid.cpp): error reporting, the per-(thread, device) library context, and the per-cell
// constant builder.  Not part of the ABI.
#pragma once
#include <hip/hip_runtime.h>

#include <cstddef>
#include <cstdint>
#include <vector>

#include "../../include/dcor.h"
#include "dcor_engine.h"

namespace dcor {
struct SignPartial;
namespace host {

// Record the message of a failure for dcor_last_error() (thread-local) and return `code`.
int fail(int code, const char* fmt, ...);
int hip_fail(hipError_t e, const char* what);
#define HIPCHK(expr)                                   \
  do {                                                 \
    hipError_t e_ = (expr);                            \
    if (e_ != hipSuccess) return hip_fail(e_, #expr);  \
  } while (0)

// DCOR_EFORK in a process forked after its parent used the engine, DCOR_ENODEV without a GPU.
int need_device();
double r_min(double a, double b);
double r_max(double a, double b);

struct Arena { void* p = nullptr; size_t bytes = 0; };
// s: the auxiliary stream of the two-stream pipelines (fork / join with the caller's stream).  The
// one-pass sign path runs its chunks on two library streams (s2, s) instead: entry marks the
// caller's stream at the call, end[] the two library streams at its end, and sig the scratch layout
// of the last call that ran there (0: the arena's last user was the caller's stream).
struct Pipe {
  hipStream_t s = nullptr, s2 = nullptr;
  hipEvent_t fork = nullptr, join = nullptr, entry = nullptr, end[2] = {nullptr, nullptr};
  uint64_t sig = 0;
};
// Pinned host memory with the event that marks the end of the last copy that read or wrote it.
struct Pinned { void* p = nullptr; size_t bytes = 0; hipEvent_t done = nullptr; };
// The library's state for one (host thread, device): scratch arenas, the auxiliary stream of the
// two-stream chunk pipeline, and pinned staging buffers (the grid's tables, two slots used in
// turn so one upload can be in flight while the next is written; the records of a pass).
struct Ctx {
  int dev = -1;
  Arena codes, rs, grid;
  Arena gpart;                    // the grid's accumulate block partials (multi-block cells)
  Arena out;                      // the synchronous grid entries' replicate records + accumulators
  hipStream_t work = nullptr;     // ... and their stream
  Pipe pipe;
  Pinned stage[2];
  int stage_next = 0;
  Pinned hrec;                    // a pass's records on their way to the caller's detail array
  Pinned hacc;                    // a shard's accumulators on their way to the host
  Arena rsj;                      // the R-stream jump polynomials (rsj_npoly of them)
  int rsj_npoly = 0;
};
int ctx_get(Ctx** out);          // the calling thread's context on the current device
void ctx_release_thread();       // free every context of the calling thread
int pipe_get(Pipe** out);
// Device arena of at least `bytes` (grows, never shrinks; counted by dcor_alloc_count()).
int arena_grow(Arena& a, size_t bytes, void** out);
// The codes arena of `c`: every user but the one-pass sign path's pipelined chunks hands it to
// kernels on the caller's stream, so taking it clears the pipe signature (the next sign call then
// orders its library streams after the caller's stream instead of overlapping this user's work).
int codes_arena(Ctx* c, size_t bytes, void** out);
// Pinned host buffer of at least `bytes`, after its previous copy finished (counted likewise).
int pinned_grow(Pinned& b, size_t bytes, void** out);
void count_alloc();              // one more device or pinned allocation (dcor_alloc_count)
// Stop the grid's persistent device workers (dcor_shutdown); `forked`: forget them unjoined.
void grid_workers_stop(bool forked);

// MT19937 jump-ahead (dcor_mtjump.cpp): the degree of the characteristic polynomial found by
// Berlekamp-Massey (19937); the cached table of nseg polynomials x^((s + 1) L - 624) mod phi,
// words 64-bit words each (copied into `table`); the host-side jumped window (test reference).
int mt_charpoly_degree();
int mt_segment_polys(int64_t L, int nseg, std::vector<uint64_t>& table, int* words);
int mt_jump_window(int32_t seed, int64_t J, uint32_t out[624]);

// All constants of one fused cell and the kernel family that runs it.
struct CellPlan {
  int kind;        // GridKind
  int dgp;         // DCOR_DGP_*
  bool nan_dgp;    // gen_bounded_factor with rho outside [0, 1]: every estimate NaN
  int vpl32;       // the sign epilogue's wave-select width (nsim > 1024)
  SignConst sign;  // family SIGN (rep_begin 0)
  SubgConst subg;  // family SUBG (rep_begin 0)
};
int prepare_cell(const dcor_cell& c, CellPlan& p);

}  // namespace host
}  // namespace dcor
