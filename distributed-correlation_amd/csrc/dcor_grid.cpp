// dcor_grid.cpp -- the grid driver of the C-ABI: every cell of an (n, rho, eps, dgp) grid in a
// few batched launches per device, sharded over the GPUs of one node.
//
// Replaces the reference's expand.grid + parallel::mclapply(run_sim_one) blocks
// (vert-cor.R:486-554; ver-cor-subG.R:245-296).  The reference runs one cell per forked worker;
// here a cell's replicates are work items: the items of all cells of one kernel family go into
// the same launches (constants from a per-launch device table), so a grid of small cells fills
// the GPU as well as one large cell does, and a 144-cell grid costs a handful of launches instead
// of 3 per cell.  Accumulators come from one segmented kernel and reach the host in one copy.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <cstring>
#include <map>
#include <string>
#include <thread>
#include <tuple>
#include <vector>

#include "../../include/dcor.h"
#include "dcor_engine.h"
#include "dcor_host.h"

using namespace dcor;
using namespace dcor::host;

namespace {

size_t al256(size_t b) { return (b + 255) & ~(size_t)255; }

// One launch group: the cells of one kernel family, DGP and epilogue width, their constant
// table, and their replicates as work items in chunks that fit the scratch budget.
struct Group {
  int kind = 0, dgp = 0, vpl32 = 0;
  std::vector<SignConst> sign;
  std::vector<SubgConst> subg;
  std::vector<GridItem> items;
  std::vector<size_t> chunk_begin;        // item index where each chunk starts (+ end sentinel)
  std::vector<uint64_t> chunk_scratch;    // scratch elements each chunk needs
  size_t tab_off = 0, item_off = 0;       // byte offsets in the uploaded table block
};

uint64_t item_scratch(int kind, int64_t n) {
  // code slabs start on 256-B boundaries (the kernels move records 16 B at a time)
  if (kind == GK_SIGN_CODES) return ((uint64_t)n + 63) & ~(uint64_t)63;   // u32 records
  if (kind == GK_SIGN_BERN) return (uint64_t)3 * 4 * ((n + 255) / 256);  // u64 plane words
  return 0;
}

size_t env_mb(const char* name, size_t dflt) {
  const char* e = std::getenv(name);
  const long v = e ? std::atol(e) : 0;
  return v > 0 ? (size_t)v << 20 : dflt;
}

struct Layout {           // the grid arena: tables | sums + partials (x2) | accumulate partials
  size_t tables = 0, sums = 0, accp = 0, total = 0;
};

}  // namespace

extern "C" {

int dcor_grid_launch(const dcor_cell* cells, int ncells, const int64_t* rep_begin,
                     const int64_t* rep_count, dcor_rep_out* d_out, dcor_accum* d_acc,
                     void* stream) {
  if (ncells < 0 || (ncells > 0 && (!cells || !rep_begin || !rep_count || !d_acc)))
    return fail(DCOR_EINVAL, "grid_launch: bad arguments");
  if (ncells == 0) return DCOR_OK;
  if (ncells > 65535) return fail(DCOR_EINVAL, "grid_launch: at most 65535 cells per launch");
  if (int st = need_device()) return st;
  const hipStream_t st0 = (hipStream_t)stream;
  // ---- plan: constants per cell, output offsets, launch groups
  std::vector<CellPlan> plan((size_t)ncells);
  std::vector<int64_t> off((size_t)ncells + 1, 0);
  for (int i = 0; i < ncells; ++i) {
    const int64_t b = rep_begin[i], c = rep_count[i];
    if (b < 0 || c < 0 || b + c > 0xffffffffLL)
      return fail(DCOR_EINVAL, "grid_launch: cell %d: replicate range must lie in [0, 2^32)", i);
    if (int st = prepare_cell(cells[i], plan[(size_t)i])) {
      char msg[512];
      dcor_last_error(msg, sizeof msg);
      return fail(st, "cell %d: %s", i, msg);
    }
    off[(size_t)i + 1] = off[(size_t)i] + c;
  }
  if (off[(size_t)ncells] > 0 && !d_out) return fail(DCOR_EINVAL, "grid_launch: null d_out");
  std::map<std::tuple<int, int, int>, Group> groups;
  std::vector<int> order((size_t)ncells);
  for (int i = 0; i < ncells; ++i) order[(size_t)i] = i;
  // longest first inside every launch: the big replicates start early, the small ones fill in
  std::stable_sort(order.begin(), order.end(), [&](int a, int b) { return cells[a].n > cells[b].n; });
  for (int i : order) {
    const CellPlan& p = plan[(size_t)i];
    if (p.nan_dgp || rep_count[i] == 0) continue;
    Group& g = groups[std::make_tuple(p.kind, p.dgp, p.vpl32)];
    g.kind = p.kind; g.dgp = p.dgp; g.vpl32 = p.vpl32;
    const uint32_t ci = (uint32_t)(p.kind == GK_SUBG ? g.subg.size() : g.sign.size());
    if (p.kind == GK_SUBG) g.subg.push_back(p.subg); else g.sign.push_back(p.sign);
    for (int64_t r = 0; r < rep_count[i]; ++r)
      g.items.push_back(GridItem{ci, (uint32_t)(rep_begin[i] + r), 0, (uint64_t)(off[(size_t)i] + r)});
  }
  // ---- chunks: the code slabs (two, for the two-stream pipeline) and Bernoulli planes
  int64_t max_n = 1;
  for (int i = 0; i < ncells; ++i) max_n = std::max<int64_t>(max_n, cells[i].n);
  size_t budget = env_mb("DCOR_GRID_SLAB_MB", (size_t)1 << 30);
  budget = std::max(budget, (size_t)1024 * (size_t)max_n * 4);
  budget = std::min(budget, (size_t)8 << 30);
  const size_t budget_el = budget / 4;   // u32 elements (u64 plane words count twice)
  size_t max_chunk_items = 1, max_scr_b = 0, ncodes_chunks = 0;
  for (auto& kv : groups) {
    Group& g = kv.second;
    const int64_t unit = (g.kind == GK_SIGN_BERN) ? 2 : 1;
    g.chunk_begin.push_back(0);
    uint64_t used = 0;
    for (size_t t = 0; t < g.items.size(); ++t) {
      const int64_t n = (g.kind == GK_SUBG) ? g.subg[g.items[t].cell].n : g.sign[g.items[t].cell].n;
      const uint64_t need = item_scratch(g.kind, n);
      const size_t in_chunk = t - g.chunk_begin.back();
      if (in_chunk > 0 && ((used + need) * unit > budget_el || in_chunk >= 0x7fffffff / 4)) {
        g.chunk_scratch.push_back(used);
        g.chunk_begin.push_back(t);
        used = 0;
      }
      g.items[t].scratch = used;
      used += need;
    }
    g.chunk_scratch.push_back(used);
    g.chunk_begin.push_back(g.items.size());
    for (size_t q = 0; q + 1 < g.chunk_begin.size(); ++q) {
      max_chunk_items = std::max(max_chunk_items, g.chunk_begin[q + 1] - g.chunk_begin[q]);
      max_scr_b = std::max(max_scr_b, (size_t)(g.chunk_scratch[q] * (g.kind == GK_SIGN_BERN ? 8 : 4)));
    }
    if (g.kind == GK_SIGN_CODES) ncodes_chunks += g.chunk_begin.size() - 1;
  }
  // ---- the table block: per group its constants and items; then the accumulate segments
  size_t tb = 0;
  for (auto& kv : groups) {
    Group& g = kv.second;
    g.tab_off = tb;
    tb += al256(g.kind == GK_SUBG ? g.subg.size() * sizeof(SubgConst) : g.sign.size() * sizeof(SignConst));
    g.item_off = tb;
    tb += al256(g.items.size() * sizeof(GridItem));
  }
  const size_t seg_off_b = tb;
  tb += al256((size_t)ncells * 8);
  const size_t seg_cnt_b = tb;
  tb += al256((size_t)ncells * 8);
  const size_t rho_b = tb;
  tb += al256((size_t)ncells * 8);
  int max_nb = 1;
  for (int i = 0; i < ncells; ++i) max_nb = std::max(max_nb, accumulate_blocks(rep_count[i]));
  Layout L;
  L.tables = 0;
  L.sums = al256(tb);
  const size_t sums_one = al256(max_chunk_items * (SIGN_SUMS * sizeof(double) + 48));
  L.accp = L.sums + 2 * sums_one;
  L.total = L.accp + al256((size_t)ncells * (size_t)max_nb * 2 * sizeof(dcor_accum));
  Ctx* ctx = nullptr;
  if (int st = ctx_get(&ctx)) return st;
  void* garena = nullptr;
  if (int st = arena_grow(ctx->grid, L.total, &garena)) return st;
  const bool two = ncodes_chunks > 1 && !(std::getenv("DCOR_SIGN_PIPELINE") &&
                                         std::strcmp(std::getenv("DCOR_SIGN_PIPELINE"), "0") == 0);
  void* scr = nullptr;
  const size_t slab_one = al256(max_scr_b);
  if (max_scr_b > 0)
    if (int st = arena_grow(ctx->codes, (two ? 2 : 1) * slab_one, &scr)) return st;
  // ---- upload the tables through the pinned staging buffer (reused once its last copy ran)
  if (ctx->staging_bytes < tb) {
    if (ctx->staging_free) HIPCHK(hipEventSynchronize(ctx->staging_free));
    if (ctx->staging) HIPCHK(hipHostFree(ctx->staging));
    ctx->staging = nullptr;
    ctx->staging_bytes = 0;
    HIPCHK(hipHostMalloc(&ctx->staging, tb, hipHostMallocDefault));
    ctx->staging_bytes = tb;
  }
  if (!ctx->staging_free) HIPCHK(hipEventCreateWithFlags(&ctx->staging_free, hipEventDisableTiming));
  HIPCHK(hipEventSynchronize(ctx->staging_free));
  char* hs = (char*)ctx->staging;
  for (auto& kv : groups) {
    const Group& g = kv.second;
    if (g.kind == GK_SUBG) std::memcpy(hs + g.tab_off, g.subg.data(), g.subg.size() * sizeof(SubgConst));
    else std::memcpy(hs + g.tab_off, g.sign.data(), g.sign.size() * sizeof(SignConst));
    std::memcpy(hs + g.item_off, g.items.data(), g.items.size() * sizeof(GridItem));
  }
  for (int i = 0; i < ncells; ++i) {
    ((int64_t*)(hs + seg_off_b))[i] = off[(size_t)i];
    ((int64_t*)(hs + seg_cnt_b))[i] = rep_count[i];
    ((double*)(hs + rho_b))[i] = cells[i].rho;
  }
  char* dg = (char*)garena;
  HIPCHK(hipMemcpyAsync(dg, hs, tb, hipMemcpyHostToDevice, st0));
  HIPCHK(hipEventRecord(ctx->staging_free, st0));
  // ---- NaN cells (gen_bounded_factor outside [0, 1]): every record NaN
  for (int i = 0; i < ncells; ++i)
    if (plan[(size_t)i].nan_dgp && rep_count[i] > 0)
      HIPCHK(hipMemsetAsync(d_out + off[(size_t)i], 0xFF, sizeof(dcor_rep_out) * (size_t)rep_count[i], st0));
  // ---- launches
  Pipe* pp = nullptr;
  hipStream_t sts[2] = {st0, st0};
  if (two) {
    if (int st = pipe_get(&pp)) return st;
    sts[1] = pp->s;
    HIPCHK(hipEventRecord(pp->fork, st0));
    HIPCHK(hipStreamWaitEvent(pp->s, pp->fork, 0));
  }
  size_t tcodes = 0;
  for (auto& kv : groups) {
    const Group& g = kv.second;
    const SignConst* dsign = (const SignConst*)(dg + g.tab_off);
    const SubgConst* dsubg = (const SubgConst*)(dg + g.tab_off);
    const GridItem* ditems = (const GridItem*)(dg + g.item_off);
    for (size_t q = 0; q + 1 < g.chunk_begin.size(); ++q) {
      const size_t b0 = g.chunk_begin[q];
      const int64_t nit = (int64_t)(g.chunk_begin[q + 1] - b0);
      int rc = 0;
      if (g.kind == GK_SIGN_CODES) {
        const int b = two ? (int)(tcodes++ & 1) : 0;
        double* sums = (double*)(dg + L.sums + (size_t)b * sums_one);
        SignPartial* part = (SignPartial*)(sums + SIGN_SUMS * max_chunk_items);
        rc = launch_grid_sign_codes(g.dgp, dsign, ditems + b0, nit,
                                    (uint32_t*)((char*)scr + (size_t)b * slab_one), sums, part,
                                    g.vpl32, d_out, sts[b]);
      } else if (g.kind == GK_SIGN_REGEN) {
        rc = launch_grid_sign_regen(g.dgp, dsign, ditems + b0, nit, d_out, st0);
      } else if (g.kind == GK_SIGN_BERN_W || g.kind == GK_SIGN_BERN) {
        SignPartial* part = (SignPartial*)(dg + L.sums);
        rc = launch_grid_sign_bern(g.kind == GK_SIGN_BERN_W, dsign, ditems + b0, nit, (uint64_t*)scr,
                                   part, g.vpl32, d_out, st0);
      } else {
        rc = launch_grid_subg(g.dgp, dsubg, ditems + b0, nit, d_out, st0);
      }
      if (rc) return hip_fail((hipError_t)rc, "grid kernel launch");
    }
  }
  if (two) {
    HIPCHK(hipEventRecord(pp->join, pp->s));
    HIPCHK(hipStreamWaitEvent(st0, pp->join, 0));
  }
  // ---- accumulators: one segmented kernel over every cell's records
  const int rc = launch_accumulate_seg(d_out, ncells, (const int64_t*)(dg + seg_off_b),
                                       (const int64_t*)(dg + seg_cnt_b), (const double*)(dg + rho_b),
                                       max_nb, (dcor_accum*)(dg + L.accp), d_acc, st0);
  if (rc) return hip_fail((hipError_t)rc, "grid accumulate launch");
  return DCOR_OK;
}

}  // extern "C"

namespace {

// One device's share of a grid: replicates [g B / G, (g+1) B / G) of every cell.
struct Shard {
  int dev = 0;
  int64_t b0 = 0, nb = 0;
  std::vector<dcor_accum> acc;
  std::vector<dcor_rep_out> rec;
  int status = DCOR_OK;
  std::string msg;
};

int run_shard(const dcor_cell* cells, int ncells, bool detail, Shard& s) {
  HIPCHK(hipSetDevice(s.dev));
  s.acc.assign((size_t)ncells * 2, dcor_accum());
  const size_t nrec = (size_t)ncells * (size_t)s.nb;
  if (detail) s.rec.resize(nrec);
  std::vector<int64_t> rb((size_t)ncells, s.b0), rn((size_t)ncells, s.nb);
  // the calling thread's stream and record buffer on this device (kept across calls)
  Ctx* ctx = nullptr;
  if (int st = ctx_get(&ctx)) return st;
  if (!ctx->work) HIPCHK(hipStreamCreateWithFlags(&ctx->work, hipStreamNonBlocking));
  const hipStream_t st = ctx->work;
  const size_t rec_b = al256(std::max<size_t>(nrec, 1) * sizeof(dcor_rep_out));
  void* buf = nullptr;
  if (int e = arena_grow(ctx->out, rec_b + (size_t)ncells * 2 * sizeof(dcor_accum), &buf)) return e;
  dcor_rep_out* d_out = (dcor_rep_out*)buf;
  dcor_accum* d_acc = (dcor_accum*)((char*)buf + rec_b);
  if (int e = dcor_grid_launch(cells, ncells, rb.data(), rn.data(), d_out, d_acc, st)) return e;
  HIPCHK(hipMemcpyAsync(s.acc.data(), d_acc, s.acc.size() * sizeof(dcor_accum), hipMemcpyDeviceToHost, st));
  if (detail && nrec)
    HIPCHK(hipMemcpyAsync(s.rec.data(), d_out, nrec * sizeof(dcor_rep_out), hipMemcpyDeviceToHost, st));
  HIPCHK(hipStreamSynchronize(st));
  return DCOR_OK;
}

}  // namespace

extern "C" {

int dcor_grid_run_multi(const dcor_cell* cells, int ncells, int64_t B, const int* device_ids,
                        int ndev, dcor_accum* h_acc, dcor_rep_out* h_detail) {
  if (!cells || ncells < 0 || B < 1 || !h_acc || ndev < 0 || (ndev > 0 && !device_ids))
    return fail(DCOR_EINVAL, "bad grid arguments");
  if (int st = need_device()) return st;
  int nvis = 0;
  HIPCHK(hipGetDeviceCount(&nvis));
  std::vector<int> devs;
  if (ndev == 0) for (int d = 0; d < nvis; ++d) devs.push_back(d);
  else devs.assign(device_ids, device_ids + ndev);
  for (int d : devs)
    if (d < 0 || d >= nvis) return fail(DCOR_EINVAL, "grid: device id %d not visible (%d devices)", d, nvis);
  if ((int64_t)devs.size() > B) devs.resize((size_t)B);   // every shard holds a replicate
  const int G = (int)devs.size();
  std::vector<Shard> sh((size_t)G);
  for (int g = 0; g < G; ++g) {
    sh[(size_t)g].dev = devs[(size_t)g];
    sh[(size_t)g].b0 = B * g / G;
    sh[(size_t)g].nb = B * (g + 1) / G - B * g / G;
  }
  const bool detail = h_detail != nullptr;
  int cur = 0;
  HIPCHK(hipGetDevice(&cur));
  if (G == 1) {  // one device: the calling thread, whose context persists across calls
    Shard& s = sh[0];
    s.status = run_shard(cells, ncells, detail, s);
    (void)hipSetDevice(cur);
    if (s.status) return s.status;
  } else {       // one host thread per shard (several may share a device), each with its own
                 // streams and scratch, released when it finishes
    std::vector<std::thread> th;
    for (int g = 0; g < G; ++g)
      th.emplace_back([&, g] {
        Shard& s = sh[(size_t)g];
        s.status = run_shard(cells, ncells, detail, s);
        if (s.status) {
          char m[512];
          dcor_last_error(m, sizeof m);
          s.msg = m;
        }
        ctx_release_thread();
      });
    for (auto& t : th) t.join();
    for (const Shard& s : sh)
      if (s.status) return fail(s.status, "grid shard on device %d: %s", s.dev, s.msg.c_str());
  }
  // rank-ordered merge (shard 0 first): deterministic for a given device list
  for (int i = 0; i < 2 * ncells; ++i) {
    h_acc[i] = sh[0].acc[(size_t)i];
    for (int g = 1; g < G; ++g) dcor_accum_merge(&h_acc[i], &sh[(size_t)g].acc[(size_t)i]);
  }
  if (detail)
    for (const Shard& s : sh)
      for (int i = 0; i < ncells; ++i)
        if (s.nb)
          std::memcpy(h_detail + (size_t)i * (size_t)B + (size_t)s.b0, s.rec.data() + (size_t)i * (size_t)s.nb,
                      (size_t)s.nb * sizeof(dcor_rep_out));
  return DCOR_OK;
}

int dcor_grid_run(const dcor_cell* cells, int ncells, int64_t B, dcor_accum* h_acc,
                  dcor_rep_out* h_detail) {
  if (int st = need_device()) return st;
  int cur = 0;
  HIPCHK(hipGetDevice(&cur));
  return dcor_grid_run_multi(cells, ncells, B, &cur, 1, h_acc, h_detail);
}

}  // extern "C"
