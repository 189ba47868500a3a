// Library identification and the thread-local error channel of the C ABI (include/gr_amd.h).
#include <atomic>
#include <cstring>
#include <string>

#include "gr_common.h"

namespace gr {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
void clear_error() { g_last_error.clear(); }

// Options: rq_fused (1: fused persistent encode kernel when the shape allows, 0: layer-wise path;
// bitwise the same IDs).
static std::atomic<int64_t> g_rq_fused{1};
// sas_fused (1: register-resident fused SASRec forward when n <= 64 and d <= 64, 0: layer-wise).
static std::atomic<int64_t> g_sas_fused{1};
// topk_sample (1: gr_score_topk_f32 takes its threshold from a strided sample pass when the
// catalog is long enough, 0: always one pass).  Same results either way; used for A/B timing.
static std::atomic<int64_t> g_topk_sample{1};
// score_flags (1: the scoring kernel's compute and store waves hand chunks over through LDS words,
// 0: one workgroup barrier per chunk).  Same results either way; used for A/B timing.
static std::atomic<int64_t> g_score_flags{1};
// score_ubmajor (1: the workgroups one XCD runs share a user block and sweep the catalog, 0: they
// share a catalog slice across all user blocks).  Same results; A/B timing.
static std::atomic<int64_t> g_score_ubmajor{1};
// score_impl (0: compute / store wave specialisation with the LDS ring, 1: direct accumulator
// stores, two workgroups per CU, 2: direct when the logits rows are 128-B line aligned, else the
// ring).  Same results.
static std::atomic<int64_t> g_score_impl{2};
// topk_wg_per_cu (0: the launch plan's own rule; 1..4: catalog slices sized for that many
// workgroups per CU).  Same results; A/B timing.
static std::atomic<int64_t> g_topk_wg_per_cu{0};
// attn_pair (1: full-sequence attention launches use the paired-tile kernel, 0 (default): the rounds-of-4
// kernel).  Same instruction sequence per row; A/B timing.
static std::atomic<int64_t> g_attn_pair{0};
// sas_rowtile (1: d = 128 layer-wise forwards fuse everything between attention launches into
// row-tile kernels, sasrec_rowtile.hip; 0: one kernel per op).  A/B timing and a second path.
static std::atomic<int64_t> g_sas_rowtile{1};
// rq_split (1: a quantize workgroup's c % 4 leftover item tiles are split into code quarters, one
// per SIMD, so the SIMDs' loads differ by at most a quarter tile; 0: round-robin tiles over waves).
static std::atomic<int64_t> g_rq_split{1};
// score_slice_major (direct-store scoring: 1 = an XCD's workgroups share catalog slices across
// user blocks (default: 255 vs 261 us at C3, scripts/ab_opt.py), 0 = they share a user block).
static std::atomic<int64_t> g_score_slice_major{1};
// attn_occ1 (hd 128 attention: 1 = one workgroup per CU, 512 registers; 0 = two, 256 registers
// with a few spills).  Identical results; A/B timing.
static std::atomic<int64_t> g_attn_occ1{0};
// attn_alt (1 (default): the attention kernel's wave -> query-tile order alternates between rounds,
// balancing the causal work over the waves; 0: ascending in every round)
static std::atomic<int64_t> g_attn_alt{1};
// attn_lazy (hd 128 attention: 1 = lazy softmax rescaling + masks on the diagonal / last tile only)
static std::atomic<int64_t> g_attn_lazy{1};
// topk_impl (1 (default): gr_score_topk_f32 = tile-max counting pass + select/re-score kernel;
// 0: sample pass + exact list pass + merges)
static std::atomic<int64_t> g_topk_impl{1};
// topk_half (tile design: 1 = the tile pass records the max of every 16-row half tile and the select
// kernel re-scores half tiles; 0 = 32-row tiles; 2 (default) = half tiles where the re-scored bytes
// saved exceed the extra maxima traffic: catalogs below ~3,700 chunks per 128 features).  Bitwise
// the same results.
static std::atomic<int64_t> g_topk_half{2};
// rt_w8 (1 (default): the post-attention row tile runs 8 waves per 64-row tile; 0: 4 waves)
static std::atomic<int64_t> g_rt_w8{1};
// lin_w8 (1 (default): gr_linear_f32's 128x128 / 128x64 tiles run 8 waves per workgroup; 0: 4)
static std::atomic<int64_t> g_lin_w8{1};
// lin_wres (1 (default): gr_linear_f32 with k = 128, n % 128 == 0, no residual and m >= 96 x 256
// runs the persistent kernel that keeps 32-column slices of w resident in registers; 0: the tiled
// kernel).  Bitwise the same results; A/B timing.
static std::atomic<int64_t> g_lin_wres{1};
// rq_pieces (1 (default): the fused encoder's tiles past q x grid run as feature-half pieces on
// twice as many workgroups plus a layers-2-3 kernel; 0: a one-tile pass on r workgroups).  Bitwise
// the same z; A/B timing.
static std::atomic<int64_t> g_rq_pieces{1};
// emb_proj (1 (default): the d = 128 forward's block 0 runs embed + LN_a0 + in-projection as one
// persistent kernel; 0: embed_ln then gr_linear_f32) and emb_rows (32 (default) or 64 rows per tile
// of that kernel).  Bitwise the same results; A/B timing.
static std::atomic<int64_t> g_emb_proj{1};
static std::atomic<int64_t> g_emb_rows{32};
// rt_kv2 (1 (default): post_attn's next-block projection with nout / 32 a multiple of 8 runs one
// column tile per wave over both row tiles (one weight stream, two chains); 0: one 32 x 32 tile
// per task).  Bitwise the same; A/B timing.
static std::atomic<int64_t> g_rt_kv2{1};
// tail_h (a last-position forward's final block: 2 (default): the one-query tail on LN_a(X) in one
// pass over its rows with an online softmax per lane group and the GEMV weights loaded a phase
// ahead (sas_tail_h2_kernel, 48 -> 39 us per C5 call); 1: the two-pass form sas_tail_h_kernel (q . K_j
// and p . V reassociated through W_k / W_v, no K|V projection of the B n rows); 0: K|V projected for
// sas_tail_kernel).  Within the logits tolerance; A/B timing.
static std::atomic<int64_t> g_tail_h{2};
// fused_tail_h (1 (default): the fused d <= 64 forward's final block of a last-position forward
// in the same H form, no K / V projection of the n tokens; 0: K and V projected).  Within the
// logits tolerance, not bitwise to 0.
static std::atomic<int64_t> g_fused_tail_h{1};
// attn_wave (6 (default): causal attention at hd 64 / 128 on a persistent grid of one wave per SIMD,
// each walking a static longest-first list of (sequence, head, query tile) items with the next
// item's Q / K / V loaded under the current item's last step (attn.hip attn_persist_kernel); 1:
// one wave per item, longest tiles first (attn_wave_kernel); 3: 1 when B * heads < 512, else 0;
// 0: the 4-wave workgroup kernel).  Bitwise the same output.
static std::atomic<int64_t> g_attn_wave{6};

int64_t option(const char* name) {
  if (!strcmp(name, "rq_fused")) return g_rq_fused.load();
  if (!strcmp(name, "sas_fused")) return g_sas_fused.load();
  if (!strcmp(name, "topk_sample")) return g_topk_sample.load();
  if (!strcmp(name, "score_flags")) return g_score_flags.load();
  if (!strcmp(name, "score_ubmajor")) return g_score_ubmajor.load();
  if (!strcmp(name, "score_impl")) return g_score_impl.load();
  if (!strcmp(name, "topk_wg_per_cu")) return g_topk_wg_per_cu.load();
  if (!strcmp(name, "attn_pair")) return g_attn_pair.load();
  if (!strcmp(name, "sas_rowtile")) return g_sas_rowtile.load();
  if (!strcmp(name, "rq_split")) return g_rq_split.load();
  if (!strcmp(name, "score_slice_major")) return g_score_slice_major.load();
  if (!strcmp(name, "attn_occ1")) return g_attn_occ1.load();
  if (!strcmp(name, "attn_alt")) return g_attn_alt.load();
  if (!strcmp(name, "attn_lazy")) return g_attn_lazy.load();
  if (!strcmp(name, "topk_impl")) return g_topk_impl.load();
  if (!strcmp(name, "topk_half")) return g_topk_half.load();
  if (!strcmp(name, "rt_w8")) return g_rt_w8.load();
  if (!strcmp(name, "lin_w8")) return g_lin_w8.load();
  if (!strcmp(name, "lin_wres")) return g_lin_wres.load();
  if (!strcmp(name, "rq_pieces")) return g_rq_pieces.load();
  if (!strcmp(name, "emb_proj")) return g_emb_proj.load();
  if (!strcmp(name, "emb_rows")) return g_emb_rows.load();
  if (!strcmp(name, "rt_kv2")) return g_rt_kv2.load();
  if (!strcmp(name, "tail_h")) return g_tail_h.load();
  if (!strcmp(name, "fused_tail_h")) return g_fused_tail_h.load();
  if (!strcmp(name, "attn_wave")) return g_attn_wave.load();
  return -1;
}
}  // namespace gr

extern "C" int gr_set_option(const char* name, int64_t value) {
  gr::clear_error();
  if (!name) return gr::fail(GR_ERR_ARG, "gr_set_option: null name");
  if (!strcmp(name, "rq_fused") && (value == 0 || value == 1)) { gr::g_rq_fused = value; return GR_OK; }
  if (!strcmp(name, "sas_fused") && (value == 0 || value == 1)) { gr::g_sas_fused = value; return GR_OK; }
  if (!strcmp(name, "topk_sample") && (value == 0 || value == 1)) { gr::g_topk_sample = value; return GR_OK; }
  if (!strcmp(name, "score_flags") && (value == 0 || value == 1)) { gr::g_score_flags = value; return GR_OK; }
  if (!strcmp(name, "score_ubmajor") && (value == 0 || value == 1)) { gr::g_score_ubmajor = value; return GR_OK; }
  if (!strcmp(name, "score_impl") && value >= 0 && value <= 4) { gr::g_score_impl = value; return GR_OK; }
  if (!strcmp(name, "topk_wg_per_cu") && value >= 0 && value <= 4) { gr::g_topk_wg_per_cu = value; return GR_OK; }
  if (!strcmp(name, "attn_pair") && (value == 0 || value == 1)) { gr::g_attn_pair = value; return GR_OK; }
  if (!strcmp(name, "sas_rowtile") && (value == 0 || value == 1)) { gr::g_sas_rowtile = value; return GR_OK; }
  if (!strcmp(name, "rq_split") && (value == 0 || value == 1)) { gr::g_rq_split = value; return GR_OK; }
  if (!strcmp(name, "score_slice_major") && (value == 0 || value == 1)) { gr::g_score_slice_major = value; return GR_OK; }
  if (!strcmp(name, "attn_occ1") && (value == 0 || value == 1)) { gr::g_attn_occ1 = value; return GR_OK; }
  if (!strcmp(name, "attn_alt") && (value == 0 || value == 1)) { gr::g_attn_alt = value; return GR_OK; }
  if (!strcmp(name, "attn_lazy") && (value == 0 || value == 1)) { gr::g_attn_lazy = value; return GR_OK; }
  if (!strcmp(name, "topk_impl") && (value == 0 || value == 1)) { gr::g_topk_impl = value; return GR_OK; }
  if (!strcmp(name, "topk_half") && value >= 0 && value <= 2) { gr::g_topk_half = value; return GR_OK; }
  if (!strcmp(name, "rt_w8") && (value == 0 || value == 1)) { gr::g_rt_w8 = value; return GR_OK; }
  if (!strcmp(name, "lin_w8") && (value == 0 || value == 1)) { gr::g_lin_w8 = value; return GR_OK; }
  if (!strcmp(name, "lin_wres") && (value == 0 || value == 1)) { gr::g_lin_wres = value; return GR_OK; }
  if (!strcmp(name, "rq_pieces") && (value == 0 || value == 1)) { gr::g_rq_pieces = value; return GR_OK; }
  if (!strcmp(name, "emb_proj") && (value == 0 || value == 1)) { gr::g_emb_proj = value; return GR_OK; }
  if (!strcmp(name, "emb_rows") && (value == 32 || value == 64)) { gr::g_emb_rows = value; return GR_OK; }
  if (!strcmp(name, "rt_kv2") && (value == 0 || value == 1)) { gr::g_rt_kv2 = value; return GR_OK; }
  if (!strcmp(name, "tail_h") && value >= 0 && value <= 2) { gr::g_tail_h = value; return GR_OK; }
  if (!strcmp(name, "fused_tail_h") && (value == 0 || value == 1)) { gr::g_fused_tail_h = value; return GR_OK; }
  if (!strcmp(name, "attn_wave") && (value == 0 || value == 1 || value == 3 || value == 6)) {
    gr::g_attn_wave = value;
    return GR_OK;
  }
  return gr::fail(GR_ERR_ARG, std::string("gr_set_option: unknown option or value: ") + name);
}

extern "C" int64_t gr_get_option(const char* name) { return name ? gr::option(name) : -1; }

extern "C" const char* gr_version(void) { return "gr_amd 0.1.0 gfx950"; }
extern "C" const char* gr_last_error(void) { return gr::g_last_error.c_str(); }
