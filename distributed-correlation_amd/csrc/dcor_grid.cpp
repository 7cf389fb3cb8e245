// dcor_grid.cpp -- the grid driver of the C-ABI: every cell of an (n, rho, eps, dgp) grid in a
// few batched launches per device, sharded over the GPUs of one node.
//
// Replaces the reference's expand.grid + parallel::mclapply(run_sim_one) blocks
// (vert-cor.R:486-554; ver-cor-subG.R:245-296).  The reference runs one cell per forked worker;
// here a cell's replicates are work items: the items of all cells of one kernel family go into
// the same launches (constants from a per-launch device table), so a grid of small cells fills
// the GPU as well as one large cell does, and a 144-cell grid costs a handful of launches instead
// of 3 per cell.
//
// Host work is O(cells + chunks), not O(replicates): a launch's items are described by pieces
// (cell, first replicate, count, first output record, first scratch element) that a device
// kernel expands into the per-workgroup item table.  Device memory is bounded whatever B is:
// items, per-replicate sums and code slabs are per chunk (a scratch budget and an item cap), and
// the synchronous entries run the replicates through a bounded record buffer in passes of whole
// accumulate blocks, so the accumulators are the same bits as one launch_accumulate per cell.
#include <hip/hip_runtime.h>
#include <unistd.h>

#include <algorithm>
#include <condition_variable>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <memory>
#include <mutex>
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

size_t env_size(const char* name, size_t dflt, int shift) {
  const char* e = dcor::variant(name);
  const long long v = e ? std::atoll(e) : 0;
  return v > 0 ? (size_t)v << shift : dflt;
}

bool codes_kind(int kind) { return kind == GK_SIGN_CODES || kind == GK_SIGN_CODES_W; }
bool subg_kind(int kind) { return kind == GK_SUBG || kind == GK_SUBG_W; }

uint64_t item_scratch(int kind, int dgp, int64_t n) {
  // code slabs (u16 records) start on 256-B boundaries: the kernels move records 16 B at a time
  if (codes_kind(kind)) return sign_item_words(n, dgp);   // u32 words
  if (kind == GK_SIGN_BERN) return (uint64_t)3 * 4 * ((n + 255) / 256);  // u64 plane words
  return 0;
}

// Replicates [rep0, rep0 + count) of cell `cell`, their records at out0, out0 + 1, ...
struct Range {
  int cell;
  int64_t rep0, count, out0;
};

// One launch group: the cells of one kernel family, DGP and epilogue width, their constant table,
// and the pieces of its chunks.
struct Group {
  int kind = 0, dgp = 0, vpl32 = 0;
  int pmax = 0;                            // largest SignConst.pieces of the group's cells
  std::vector<SignConst> sign;
  std::vector<SubgConst> subg;
  std::map<int, uint32_t> slot;            // global cell -> constant table index
  std::vector<GridPiece> pieces;
  std::vector<size_t> chunk_p;             // first piece of each chunk (+ end sentinel)
  std::vector<uint64_t> chunk_items;       // items per chunk
  std::vector<uint64_t> chunk_base;        // first item of each chunk in the exec's item table
  size_t tab_off = 0;                      // byte offset of the constants in the uploaded block
};

// The kernels of a set of ranges on `st0` (plus the context's auxiliary stream for the one-pass
// sign chunks).  Records go to d_out[range.out0 + r].  The tables travel through the context's
// pinned staging slots; `extra` bytes (accumulate tables) are appended to the same upload and
// their device address returned in *extra_dev.
int exec_ranges(const dcor_cell* cells, const std::vector<CellPlan>& cp, const std::vector<Range>& ranges,
                dcor_rep_out* d_out, hipStream_t st0, Ctx* ctx, const void* extra, size_t extra_b,
                void** extra_dev) {
  // ---- groups, in the order of their first range (longest n first inside a launch, see below)
  std::map<std::tuple<int, int, int>, Group> groups;
  std::vector<int> order;
  for (size_t q = 0; q < ranges.size(); ++q) order.push_back((int)q);
  // longest first inside every launch: the big replicates start early, the small ones fill in
  std::stable_sort(order.begin(), order.end(),
                   [&](int a, int b) { return cells[ranges[a].cell].n > cells[ranges[b].cell].n; });
  const size_t item_cap = env_size("DCOR_GRID_CHUNK_ITEMS", (size_t)1 << 19, 0);
  int64_t max_n = 1;
  for (const Range& r : ranges) max_n = std::max<int64_t>(max_n, cells[r.cell].n);
  size_t budget = env_size("DCOR_GRID_SLAB_MB", (size_t)1 << 30, 20);
  budget = std::max(budget, (size_t)1024 * (size_t)max_n * 4);
  budget = std::min(budget, (size_t)8 << 30);
  const uint64_t budget_el = budget / 4;   // u32 elements (u64 plane words count twice)
  // chunk state per group while pieces are laid out
  struct Fill { uint64_t items = 0, used = 0; };
  std::map<std::tuple<int, int, int>, Fill> fill;
  // per-group chunk limits: the scratch budget and the item cap, and for the one-pass sign
  // kernels at least DCOR_GRID_MIN_CHUNKS (default 4) equal chunks once there are 2048 items, so
  // pass 2 (latency-bound) of one chunk runs beside pass 1 (VALU-bound) of the next on the two
  // streams -- at the reference grids' n (1000-12000) pass 2 costs as much as pass 1
  struct Lim { uint64_t items = 0, scratch = 0, cap_items = 0, cap_scr = 0; };
  std::map<std::tuple<int, int, int>, Lim> lim;
  const uint64_t min_chunks = env_size("DCOR_GRID_MIN_CHUNKS", 4, 0);
  for (const Range& r : ranges) {
    const CellPlan& p = cp[(size_t)r.cell];
    if (r.count == 0 || p.nan_dgp) continue;
    Lim& l = lim[std::make_tuple(p.kind, p.dgp, p.vpl32)];
    l.items += (uint64_t)r.count;
    l.scratch += (uint64_t)r.count * item_scratch(p.kind, p.dgp, cells[r.cell].n) * (p.kind == GK_SIGN_BERN ? 2 : 1);
  }
  for (auto& kv : lim) {
    Lim& l = kv.second;
    l.cap_items = item_cap;
    l.cap_scr = budget_el;
    if (codes_kind(std::get<0>(kv.first)) && l.items >= 2048 && min_chunks > 1) {
      uint64_t nch = std::max<uint64_t>(min_chunks, (l.scratch + budget_el - 1) / budget_el);
      nch = std::max<uint64_t>(nch, (l.items + item_cap - 1) / item_cap);
      l.cap_items = std::min<uint64_t>(item_cap, (l.items + nch - 1) / nch);
    }
  }
  for (int q : order) {
    const Range& r = ranges[(size_t)q];
    const CellPlan& p = cp[(size_t)r.cell];
    if (r.count == 0) continue;
    if (p.nan_dgp) {   // gen_bounded_factor outside [0, 1]: every record NaN
      HIPCHK(hipMemsetAsync(d_out + r.out0, 0xFF, sizeof(dcor_rep_out) * (size_t)r.count, st0));
      continue;
    }
    const auto key = std::make_tuple(p.kind, p.dgp, p.vpl32);
    Group& g = groups[key];
    Fill& f = fill[key];
    if (g.chunk_p.empty()) {
      g.kind = p.kind; g.dgp = p.dgp; g.vpl32 = p.vpl32;
      g.chunk_p.push_back(0);
    }
    auto it = g.slot.find(r.cell);
    uint32_t ci;
    if (it == g.slot.end()) {
      ci = (uint32_t)(subg_kind(p.kind) ? g.subg.size() : g.sign.size());
      if (subg_kind(p.kind)) {
        g.subg.push_back(p.subg);
      } else {
        g.sign.push_back(p.sign);
        g.pmax = std::max<int>(g.pmax, p.sign.pieces);
      }
      g.slot[r.cell] = ci;
    } else {
      ci = it->second;
    }
    const int64_t n = cells[r.cell].n;
    const uint64_t need = item_scratch(p.kind, p.dgp, n);
    const uint64_t unit = (p.kind == GK_SIGN_BERN) ? 2 : 1;
    const Lim& lm = lim[key];
    int64_t done = 0;
    while (done < r.count) {
      uint64_t fit = (uint64_t)(r.count - done);
      fit = std::min<uint64_t>(fit, lm.cap_items - f.items);
      if (need) fit = std::min<uint64_t>(fit, (lm.cap_scr / unit - f.used) / need);
      if (fit == 0) {   // chunk full: close it (a fresh chunk always takes >= 1024 items)
        if (f.items == 0) return fail(DCOR_EINVAL, "grid: a replicate of cell %d exceeds the scratch budget", r.cell);
        g.chunk_items.push_back(f.items);
        g.chunk_p.push_back(g.pieces.size());
        f = Fill();
        continue;
      }
      g.pieces.push_back(GridPiece{ci, (uint32_t)(r.rep0 + done), f.items, fit, (uint64_t)(r.out0 + done),
                                   f.used, need});
      f.items += fit;
      f.used += fit * need;
      done += (int64_t)fit;
    }
  }
  size_t max_scr_b = 0, max_sums_b = 0, ncodes_chunks = 0;
  uint64_t tot_items = 0;   // every chunk's items, one table expanded by one launch
  std::vector<GridPiece> all_pieces;
  for (auto& kv : groups) {
    Group& g = kv.second;
    const Fill& f = fill[kv.first];
    if (f.items) {
      g.chunk_items.push_back(f.items);
      g.chunk_p.push_back(g.pieces.size());
    }
    for (size_t c = 0; c + 1 < g.chunk_p.size(); ++c) {
      const uint64_t ni = g.chunk_items[c];
      g.chunk_base.push_back(tot_items);
      for (size_t q = g.chunk_p[c]; q < g.chunk_p[c + 1]; ++q) {
        GridPiece pc = g.pieces[q];
        pc.item0 += tot_items;
        all_pieces.push_back(pc);
      }
      tot_items += ni;
      uint64_t used = 0;
      for (size_t q = g.chunk_p[c]; q < g.chunk_p[c + 1]; ++q) used += g.pieces[q].count * g.pieces[q].scr_stride;
      max_scr_b = std::max<size_t>(max_scr_b, used * (g.kind == GK_SIGN_BERN ? 8 : 4));
      if (g.kind == GK_SIGN_CODES)
        max_sums_b = std::max<size_t>(max_sums_b, ni * (SIGN_SUMS * sizeof(double) + SIGN_PARTIAL_BYTES));
      else if (g.kind == GK_SIGN_CODES_W)   // the partials too (the unfused wave pass 2)
        max_sums_b = std::max<size_t>(max_sums_b, ni * (SIGN_SUMS * sizeof(double) + SIGN_PARTIAL_BYTES));
      else if (g.kind == GK_SIGN_BERN || g.kind == GK_SIGN_BERN_W)
        max_sums_b = std::max<size_t>(max_sums_b, ni * SIGN_PARTIAL_BYTES);
    }
    if (codes_kind(g.kind)) ncodes_chunks += g.chunk_p.size() - 1;
  }
  // ---- the table block: per group its constants; every piece; then the caller's extra tables
  size_t tb = 0;
  for (auto& kv : groups) {
    Group& g = kv.second;
    g.tab_off = tb;
    tb += al256(subg_kind(g.kind) ? g.subg.size() * sizeof(SubgConst) : g.sign.size() * sizeof(SignConst));
  }
  const size_t piece_off = tb;
  tb += al256(all_pieces.size() * sizeof(GridPiece));
  const size_t extra_off = tb;
  tb += al256(extra_b);
  tb = std::max<size_t>(tb, 256);
  const bool two = ncodes_chunks > 1 && !(dcor::variant("DCOR_SIGN_PIPELINE") &&
                                         std::strcmp(dcor::variant("DCOR_SIGN_PIPELINE"), "0") == 0);
  const int nslot = two ? 2 : 1;
  const size_t sums_one = al256(std::max<size_t>(max_sums_b, 8));
  const size_t items_off = al256(tb), sums_off = items_off + al256(std::max<uint64_t>(tot_items, 1) * sizeof(GridItem));
  const size_t total = sums_off + (size_t)nslot * sums_one;
  void* garena = nullptr;
  if (int st = arena_grow(ctx->grid, total, &garena)) return st;
  void* scr = nullptr;
  const size_t slab_one = al256(max_scr_b) + 256;   // + pass 2's 16-B over-read past the last record
  if (max_scr_b > 0)
    if (int st = codes_arena(ctx, (size_t)nslot * slab_one, &scr)) return st;
  // ---- upload through a pinned staging slot (its previous upload finished long ago in steady
  // state: the slots alternate, and each synchronous call ends with a stream sync)
  Pinned& stg = ctx->stage[ctx->stage_next];
  ctx->stage_next ^= 1;
  void* hsv = nullptr;
  if (int st = pinned_grow(stg, tb, &hsv)) return st;
  char* hs = (char*)hsv;
  for (auto& kv : groups) {
    const Group& g = kv.second;
    if (subg_kind(g.kind)) std::memcpy(hs + g.tab_off, g.subg.data(), g.subg.size() * sizeof(SubgConst));
    else std::memcpy(hs + g.tab_off, g.sign.data(), g.sign.size() * sizeof(SignConst));
  }
  std::memcpy(hs + piece_off, all_pieces.data(), all_pieces.size() * sizeof(GridPiece));
  if (extra_b) std::memcpy(hs + extra_off, extra, extra_b);
  char* dg = (char*)garena;
  HIPCHK(hipMemcpyAsync(dg, hs, tb, hipMemcpyHostToDevice, st0));
  HIPCHK(hipEventRecord(stg.done, st0));
  if (extra_dev) *extra_dev = dg + extra_off;
  // ---- launches: one expansion of every chunk's items, then per chunk the family's kernels
  GridItem* items_all = (GridItem*)(dg + items_off);
  if (int rc = launch_grid_expand((const GridPiece*)(dg + piece_off), (int64_t)all_pieces.size(), items_all, st0))
    return hip_fail((hipError_t)rc, "grid item expansion");
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
    for (size_t c = 0; c + 1 < g.chunk_p.size(); ++c) {
      const int64_t nit = (int64_t)g.chunk_items[c];
      const int b = (two && codes_kind(g.kind)) ? (int)(tcodes++ & 1) : 0;
      const GridItem* items = items_all + g.chunk_base[c];
      char* sums = dg + sums_off + (size_t)b * sums_one;
      int rc = 0;
      if (g.kind == GK_SIGN_CODES_W) {
        rc = launch_grid_sign_codes_w(g.dgp, dsign, items, nit, (uint32_t*)((char*)scr + (size_t)b * slab_one),
                                      (double*)sums, g.vpl32, g.pmax, d_out, sts[b]);
      } else if (g.kind == GK_SIGN_CODES) {
        rc = launch_grid_sign_codes(g.dgp, dsign, items, nit, (uint32_t*)((char*)scr + (size_t)b * slab_one),
                                    (double*)sums, (SignPartial*)(sums + SIGN_SUMS * sizeof(double) * (size_t)nit),
                                    g.vpl32, g.pmax, d_out, sts[b]);
      } else if (g.kind == GK_SIGN_REGEN) {
        rc = launch_grid_sign_regen(g.dgp, dsign, items, nit, d_out, st0);
      } else if (g.kind == GK_SIGN_BERN_W || g.kind == GK_SIGN_BERN) {
        rc = launch_grid_sign_bern(g.kind == GK_SIGN_BERN_W, dsign, items, nit, (uint64_t*)scr,
                                   (SignPartial*)sums, g.vpl32, d_out, st0);
      } else if (g.kind == GK_SUBG_W) {
        rc = launch_grid_subg_w(g.dgp, dsubg, items, nit, g.vpl32, d_out, st0);
      } else {
        rc = launch_grid_subg(g.dgp, dsubg, items, nit, d_out, st0);
      }
      if (rc) return hip_fail((hipError_t)rc, "grid kernel launch");
    }
  }
  if (two) {
    HIPCHK(hipEventRecord(pp->join, pp->s));
    HIPCHK(hipStreamWaitEvent(st0, pp->join, 0));
  }
  return DCOR_OK;
}

int plan_cells(const dcor_cell* cells, int ncells, std::vector<CellPlan>& cp) {
  cp.resize((size_t)ncells);
  for (int i = 0; i < ncells; ++i)
    if (int st = prepare_cell(cells[i], cp[(size_t)i])) {
      char msg[512];
      dcor_last_error(msg, sizeof msg);
      return fail(st, "cell %d: %s", i, msg);
    }
  return DCOR_OK;
}

// Ragged partial slots of the multi-block cells: poff[i] (or -1 for a one-block cell).
size_t partial_layout(const int64_t* count, int ncells, std::vector<int64_t>& poff,
                      std::vector<AccCell>& multi) {
  size_t np = 0;
  poff.assign((size_t)ncells, -1);
  for (int i = 0; i < ncells; ++i) {
    const int nb = accumulate_blocks(count[i]);
    if (nb > 1) {
      poff[(size_t)i] = (int64_t)np;
      multi.push_back(AccCell{count[i], (int64_t)np, i, 0});
      np += (size_t)nb;
    }
  }
  return np;
}

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
  std::vector<CellPlan> cp;
  int64_t tot = 0;
  for (int i = 0; i < ncells; ++i) {
    const int64_t b = rep_begin[i], c = rep_count[i];
    if (b < 0 || c < 0 || b + c > 0xffffffffLL)
      return fail(DCOR_EINVAL, "grid_launch: cell %d: replicate range must lie in [0, 2^32)", i);
    tot += c;
  }
  if (int st = plan_cells(cells, ncells, cp)) return st;
  if (tot > 0 && !d_out) return fail(DCOR_EINVAL, "grid_launch: null d_out");
  // one pass: every cell's records, cell-major in the caller's buffer
  std::vector<Range> ranges;
  std::vector<AccEntry> ent;
  std::vector<int64_t> poff;
  std::vector<AccCell> multi;
  const size_t np = partial_layout(rep_count, ncells, poff, multi);
  int64_t off = 0;
  for (int i = 0; i < ncells; ++i) {
    ranges.push_back(Range{i, rep_begin[i], rep_count[i], off});
    ent.push_back(AccEntry{off, 0, accumulate_blocks(rep_count[i]), rep_count[i], poff[(size_t)i],
                           cells[i].rho, i, 0});
    off += rep_count[i];
  }
  Ctx* ctx = nullptr;
  if (int st = ctx_get(&ctx)) return st;
  void* part = nullptr;
  if (np) if (int st = arena_grow(ctx->gpart, np * 2 * sizeof(dcor_accum), &part)) return st;
  const size_t ent_b = al256(ent.size() * sizeof(AccEntry));
  std::vector<char> extra(ent_b + multi.size() * sizeof(AccCell), 0);
  std::memcpy(extra.data(), ent.data(), ent.size() * sizeof(AccEntry));
  if (!multi.empty()) std::memcpy(extra.data() + ent_b, multi.data(), multi.size() * sizeof(AccCell));
  void* dextra = nullptr;
  if (int st = exec_ranges(cells, cp, ranges, d_out, st0, ctx, extra.data(), extra.size(), &dextra)) return st;
  int max_span = 1;
  for (const AccEntry& e : ent) max_span = std::max<int>(max_span, (int)(e.bhi - e.blo));
  int rc = launch_accumulate_pass(d_out, (const AccEntry*)dextra, ncells, max_span, (dcor_accum*)part, d_acc, st0);
  if (!rc && !multi.empty())
    rc = launch_accumulate_merge_cells((const AccCell*)((char*)dextra + ent_b), (int)multi.size(),
                                       (const dcor_accum*)part, d_acc, st0);
  if (rc) return hip_fail((hipError_t)rc, "grid accumulate launch");
  return DCOR_OK;
}

}  // extern "C"

namespace {

// One device's share of a grid: replicates [b0, b0 + nb) of every cell.
struct Shard {
  int dev = 0;
  int64_t b0 = 0, nb = 0;
  std::vector<dcor_accum> acc;
  int status = DCOR_OK;
  std::string msg;
};

// The shard on the calling thread's context for its device: the replicates run in passes over a
// bounded record buffer (DCOR_GRID_REC_MB, default 256 MiB); each pass holds whole accumulate
// blocks of consecutive cells, so the accumulators equal one launch_accumulate per cell.  With
// `detail`, every pass's records reach h_detail[cell * B + b0 + r] through pinned memory.
int run_shard(const dcor_cell* cells, int ncells, int64_t B, dcor_rep_out* h_detail, Shard& s) {
  HIPCHK(hipSetDevice(s.dev));
  s.acc.assign((size_t)ncells * 2, dcor_accum());
  std::vector<CellPlan> cp;
  if (int st = plan_cells(cells, ncells, cp)) return st;
  Ctx* ctx = nullptr;
  if (int st = ctx_get(&ctx)) return st;
  if (!ctx->work) HIPCHK(hipStreamCreateWithFlags(&ctx->work, hipStreamNonBlocking));
  const hipStream_t st = ctx->work;
  const int64_t nb = s.nb;
  std::vector<int64_t> counts((size_t)ncells, nb), poff;
  std::vector<AccCell> multi;
  const size_t np = partial_layout(counts.data(), ncells, poff, multi);
  const int64_t per = accumulate_per(nb), nblk = accumulate_blocks(nb);
  const int64_t pass_rec = std::max<int64_t>(
      per, (int64_t)(env_size("DCOR_GRID_REC_MB", (size_t)256 << 20, 20) / sizeof(dcor_rep_out)));
  const int64_t total = (int64_t)ncells * nb;
  const int64_t buf_rec = std::max<int64_t>(1, std::min<int64_t>(total, pass_rec));
  void* buf = nullptr;
  if (int e = arena_grow(ctx->out, al256((size_t)buf_rec * sizeof(dcor_rep_out)) + (size_t)ncells * 2 * sizeof(dcor_accum),
                         &buf)) return e;
  dcor_rep_out* d_out = (dcor_rep_out*)buf;
  dcor_accum* d_acc = (dcor_accum*)((char*)buf + al256((size_t)buf_rec * sizeof(dcor_rep_out)));
  void* part = nullptr;
  if (np) if (int e = arena_grow(ctx->gpart, np * 2 * sizeof(dcor_accum), &part)) return e;
  // passes: (cell, block) in cell-major order
  int cell = 0;
  int64_t blk = 0;
  while (cell < ncells && nb > 0) {
    std::vector<Range> ranges;
    std::vector<AccEntry> ent;
    int64_t used = 0;
    while (cell < ncells) {
      // blocks of this cell that fit the pass
      const int64_t r0 = blk * per;
      int64_t bhi = blk;
      int64_t r1 = r0;
      while (bhi < nblk) {
        const int64_t e = std::min<int64_t>((bhi + 1) * per, nb);
        if (used + (e - r0) > pass_rec && bhi > blk) break;
        if (used + (e - r0) > pass_rec && !ranges.empty()) break;
        r1 = e;
        ++bhi;
      }
      if (bhi == blk) break;   // nothing of this cell fits: next pass
      ranges.push_back(Range{cell, s.b0 + r0, r1 - r0, used});
      ent.push_back(AccEntry{used, blk, bhi, nb, poff[(size_t)cell], cells[cell].rho, cell, 0});
      used += r1 - r0;
      if (bhi == nblk) { ++cell; blk = 0; } else { blk = bhi; break; }
    }
    void* dent = nullptr;
    if (int e = exec_ranges(cells, cp, ranges, d_out, st, ctx, ent.data(), ent.size() * sizeof(AccEntry), &dent))
      return e;
    int max_span = 1;
    for (const AccEntry& e : ent) max_span = std::max<int>(max_span, (int)(e.bhi - e.blo));
    if (int rc = launch_accumulate_pass(d_out, (const AccEntry*)dent, (int)ent.size(), max_span, (dcor_accum*)part,
                                        d_acc, st))
      return hip_fail((hipError_t)rc, "grid accumulate launch");
    if (h_detail) {   // the pass's records -> pinned -> the caller's cell-major detail array
      void* hp = nullptr;
      if (int e = pinned_grow(ctx->hrec, (size_t)used * sizeof(dcor_rep_out), &hp)) return e;
      HIPCHK(hipMemcpyAsync(hp, d_out, (size_t)used * sizeof(dcor_rep_out), hipMemcpyDeviceToHost, st));
      HIPCHK(hipEventRecord(ctx->hrec.done, st));
      HIPCHK(hipEventSynchronize(ctx->hrec.done));
      for (const Range& r : ranges)
        std::memcpy(h_detail + (size_t)r.cell * (size_t)B + (size_t)r.rep0, (dcor_rep_out*)hp + r.out0,
                    (size_t)r.count * sizeof(dcor_rep_out));
    }
  }
  if (!multi.empty()) {   // the merge table rides in one more small upload
    void* hsv = nullptr;
    Pinned& stg = ctx->stage[ctx->stage_next];
    ctx->stage_next ^= 1;
    if (int e = pinned_grow(stg, multi.size() * sizeof(AccCell), &hsv)) return e;
    std::memcpy(hsv, multi.data(), multi.size() * sizeof(AccCell));
    void* dm = nullptr;
    if (int e = arena_grow(ctx->grid, al256(multi.size() * sizeof(AccCell)), &dm)) return e;
    HIPCHK(hipMemcpyAsync(dm, hsv, multi.size() * sizeof(AccCell), hipMemcpyHostToDevice, st));
    HIPCHK(hipEventRecord(stg.done, st));
    if (int rc = launch_accumulate_merge_cells((const AccCell*)dm, (int)multi.size(), (const dcor_accum*)part, d_acc, st))
      return hip_fail((hipError_t)rc, "grid accumulate merge");
  }
  if (nb > 0) {   // through pinned memory: a pageable D2H copy would stage and block
    void* ha = nullptr;
    const size_t ab = s.acc.size() * sizeof(dcor_accum);
    if (int e = pinned_grow(ctx->hacc, ab, &ha)) return e;
    HIPCHK(hipMemcpyAsync(ha, d_acc, ab, hipMemcpyDeviceToHost, st));
    HIPCHK(hipEventRecord(ctx->hacc.done, st));
    HIPCHK(hipStreamSynchronize(st));
    std::memcpy(s.acc.data(), ha, ab);
  }
  HIPCHK(hipStreamSynchronize(st));
  return DCOR_OK;
}

// Persistent per-device workers of dcor_grid_run_multi: worker (device d, k-th listing of d) is
// one host thread, so its library context -- arenas, streams, pinned buffers -- survives across
// calls; dcor_shutdown stops the workers and frees their contexts with the others.
struct Worker {
  std::thread th;
  std::mutex mu;
  std::condition_variable cv;
  std::function<void()> job;
  bool busy = false, stop = false;
  void loop() {
    for (;;) {
      std::function<void()> j;
      {
        std::unique_lock<std::mutex> lk(mu);
        cv.wait(lk, [&] { return stop || (busy && job); });
        if (stop) return;
        j = std::move(job);
        job = nullptr;
      }
      j();
      {
        std::lock_guard<std::mutex> lk(mu);
        busy = false;
      }
      cv.notify_all();
    }
  }
  void submit(std::function<void()> f) {
    std::lock_guard<std::mutex> lk(mu);
    job = std::move(f);
    busy = true;
    cv.notify_all();
  }
  void wait() {
    std::unique_lock<std::mutex> lk(mu);
    cv.wait(lk, [&] { return !busy; });
  }
};
std::mutex g_workers_mu;
// Held across the whole worker section of dcor_grid_run_multi: a worker holds one job at a time,
// so two host threads running multi-device grids at once take turns (each still runs its shards in
// parallel over its devices) instead of overwriting each other's jobs.
std::mutex g_multi_mu;
std::map<std::pair<int, int>, Worker*>* g_workers = new std::map<std::pair<int, int>, Worker*>();
int g_workers_pid = 0;

Worker* worker_get(int dev, int k) {
  std::lock_guard<std::mutex> lk(g_workers_mu);
  Worker*& w = (*g_workers)[std::make_pair(dev, k)];
  if (!w) {
    w = new Worker();
    w->th = std::thread([w] { w->loop(); });
    g_workers_pid = (int)getpid();
  }
  return w;
}

}  // namespace

namespace dcor {
namespace host {
// dcor_shutdown's first step: stop and join the grid workers (their contexts are freed with the
// rest).  In a forked child the threads do not exist: forget them without joining.
void grid_workers_stop(bool forked) {
  std::lock_guard<std::mutex> lk(g_workers_mu);
  if (forked || g_workers_pid != (int)getpid()) {
    g_workers = new std::map<std::pair<int, int>, Worker*>();   // leaked on purpose
    return;
  }
  for (auto& kv : *g_workers) {
    Worker* w = kv.second;
    {
      std::lock_guard<std::mutex> lw(w->mu);
      w->stop = true;
    }
    w->cv.notify_all();
    w->th.join();
    delete w;
  }
  g_workers->clear();
}
}  // namespace host
}  // namespace dcor

extern "C" {

int dcor_grid_run_multi(const dcor_cell* cells, int ncells, int64_t B, const int* device_ids,
                        int ndev, dcor_accum* h_acc, dcor_rep_out* h_detail) {
  if (!cells || ncells < 0 || B < 1 || !h_acc || ndev < 0 || (ndev > 0 && !device_ids))
    return fail(DCOR_EINVAL, "bad grid arguments");
  if (B > 0xffffffffLL) return fail(DCOR_EINVAL, "grid: B must be below 2^32");
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
  int cur = 0;
  HIPCHK(hipGetDevice(&cur));
  if (G == 1) {  // one device: the calling thread, whose context persists across calls
    Shard& s = sh[0];
    s.status = run_shard(cells, ncells, B, h_detail, s);
    (void)hipSetDevice(cur);
    if (s.status) return s.status;
  } else {       // one persistent worker per (device, listing): several may share a device
    std::lock_guard<std::mutex> run_lk(g_multi_mu);
    std::map<int, int> seen;
    std::vector<Worker*> ws;
    for (int g = 0; g < G; ++g) {
      Shard& s = sh[(size_t)g];
      Worker* w = worker_get(s.dev, seen[s.dev]++);
      w->submit([&, g] {
        Shard& sg = sh[(size_t)g];
        sg.status = run_shard(cells, ncells, B, h_detail, sg);
        if (sg.status) {
          char m[512];
          dcor_last_error(m, sizeof m);
          sg.msg = m;
        }
      });
      ws.push_back(w);
    }
    for (Worker* w : ws) w->wait();
    for (const Shard& s : sh)
      if (s.status) return fail(s.status, "grid shard on device %d: %s", s.dev, s.msg.c_str());
  }
  // rank-ordered merge (shard 0 first): deterministic for a given device list
  for (int i = 0; i < 2 * ncells; ++i) {
    h_acc[i] = sh[0].acc[(size_t)i];
    for (int g = 1; g < G; ++g) dcor_accum_merge(&h_acc[i], &sh[(size_t)g].acc[(size_t)i]);
  }
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
