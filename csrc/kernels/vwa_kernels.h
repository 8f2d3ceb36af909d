// Host-visible launch interface of the gfx950 kernel library (C ABI, raw pointers + hipStream_t).
// The torch binding layer (csrc/bindings.cpp) is the only caller; every launcher is
// graph-capture safe (no allocation, no synchronisation, only the given stream).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

struct SkinnyParams {
  const uint16_t* X; int ldx;
  const uint16_t* W;
  int M, N, K;
  const uint16_t* bias;
  int fuse_rms; float eps;
  void* Y; int ldy; int y_f32;
  const uint16_t* R; int ldr;
  int n_q_heads, n_kv_heads, head_dim, use_rope;
  const int* positions;
  const int64_t* slots;
  const float* rope;
  uint16_t* q_out; int ldq;
  uint16_t* k_cache; uint16_t* v_cache;
  int block_size;
  int64_t cache_stride_block, cache_stride_head, cache_stride_tok;
  const float* w_scale;  // non-null: W is OCP fp8 e4m3 [N, K] bytes with per-row scales (W8A8 path)
  int w_first;           // stream kernel: issue the first weight loads before staging X
  // fuse_rms == 2: LayerNorm folded into the GEMM (stream kernel, bf16 weights): W holds
  // W*gamma, bias holds b + W.beta, ln_c[n] = sum_k (W*gamma)[n][k]; the kernel computes each
  // row's mean/rstd from the staged X and applies y = rstd * (acc - mean * ln_c[n]) + bias
  const float* ln_c;
  // w_tiled: W (bf16) is stored pre-tiled for the MFMA B operand: for each 16-row tile T and
  // 128-wide k-group kg, a contiguous 4 KB block [s = 0..3][lane = 0..63][8 bf16] holding
  // W[16 T + (lane & 15)][128 kg + 32 (lane >> 4) + 8 s + e] -- every weight load instruction of
  // the streaming / chained kernels then reads 1 KB contiguous (ops.tile_weight)
  int w_tiled;
  // col_mask (LM head under a grammar mask, EPI store, <= 64 tiles per workgroup): u32 token
  // bitmask rows [col_mask_rows][col_mask_ld]; only the 16-column tiles holding an admissible token
  // of some row are computed, the other outputs are left unwritten (the sampler never reads a
  // masked logit).  Ignored (every tile computed) where the kernel cannot take it.
  const uint32_t* col_mask; int col_mask_ld; int col_mask_rows;
};

// Paged / strided KV addressing shared by the attention kernels:
//   addr(seq b, kv head h, token t) = base + table[b*table_stride + t/block_size]*stride_block
//                                     + h*stride_head + (t%block_size)*stride_tok
struct KVView {
  const uint16_t* k; const uint16_t* v;
  const int* block_table; int table_stride;
  int block_size;
  int64_t stride_block, stride_head, stride_tok;
};

struct DecodeAttnParams {
  const uint16_t* q; int ldq;       // [rows, n_q_heads*D]
  KVView kv;
  const int* ctx_lens;              // [rows] number of keys visible to the row
  const int* seq_ids;               // [rows] row -> block-table row
  int rows, n_q_heads, n_kv_heads, head_dim;
  float scale;
  int split_tokens;                 // keys per split workgroup
  int n_splits;                     // max splits (grid.y)
  float* part_o; float* part_ml;    // [rows][n_splits][n_q_heads][D], [rows][n_splits][n_q_heads][2]
  int* counters;                    // [rows * n_kv_heads] chunk tickets, zero between launches
  uint16_t* out; int ldo;           // [rows, n_q_heads*D]
  // optional (chained attention, <= 4 rows): the block table of each ROW's sequence, [rows][rt_stride
  // <= 128] -- read in the same round trip as seq_ids / ctx_lens (no dependent table load)
  const int* row_table; int rt_stride;
  // optional (multi-query kernel, non-chained): [P, n_real] on the device -- the first P keys (a
  // multiple of 32) of rows 0 .. n_real-1 are the SAME physical K/V (the prefix-cached prompt every
  // session shares), so those rows are grouped RG at a time across sequences for keys < P (one
  // K/V read per group instead of per sequence) and by sequence for their own keys >= P.
  const int* shared;
  // optional (chained attention): per-workgroup step plan [grid][16] int32 -- plan_mode 1: write it
  // (layer 0), 2: read it (layers 1..; mq_attention.h), 0: off
  int* plan; int plan_mode;
};

// Chained decode GEMM phases in one persistent launch (skinny_stream.hip, vwa_chain): each phase
// is a streaming-GEMM SkinnyParams + epilogue id (1 residual, 2 SwiGLU, 4 QKV, 0 store); the
// launcher fills nt / nb.  bar: >= 1536 zero-initialised bytes of monotonic ticket counters and
// the timeout flag (skinny_stream.hip chain_arrive), valid across launches.
constexpr int kChainMaxPhases = 4;
struct ChainPhase {
  SkinnyParams p;
  int epi, nt, nb;
  int xg;  // X fragments streamed with the weights (X rows do not fit LDS; set by vwa_chain_prepare)
};
// Tensor-parallel in-launch all-reduce of the chained Llama tail (world 1: off).  The row-parallel
// phases (o_proj, down) write this rank's f32 partial rows into stage[rank] (region 0 / 1); after
// a grid barrier workgroup 0 signals every peer (flag_out[p] <- round), every workgroup waits for
// all peers' signals (flag_in[p]) and reduces its slice h += sum over ranks in rank order (the
// same bits on every rank), then the next barrier.  Rounds are counted by *epoch (two per launch).
struct ChainTP {
  int world, rank;
  float* stage[8];     // each rank's chain regions (IPC-mapped), 2 x region floats
  int* flag_out[8];    // peer p's flag word for this rank
  int* flag_in;        // this rank's flag words [8] (peer p signals [p])
  int* epoch;          // this rank's round counter (private)
  int region;          // floats per region (>= M x hidden)
};

// (64-byte aligned: a multi-layer launch indexes an array of them, and each one's scalar-cache
// warm-up, chain_kernel, covers exactly its 25 lines)
struct alignas(64) ChainParams {
  ChainPhase ph[kChainMaxPhases];
  int n;
  int seq;                 // 0 Llama tail, 1 Whisper tail, 2 Whisper middle (skinny_stream.hip chain_kernel)
  int pre2;                // issue a phase's first two weight items before the barrier wait (else one)
  int next0;               // phase 1's item 0 rides in the register set a 1-item phase 0 leaves free
  int xdma;                // X staged by one wave with LDS-DMA while the others stream (chain_phase)
  int osub;                // attention launches: phase 0 only on the workgroups without an attention item
  unsigned* bar;
  int bar_mode;            // 0: flat ticket counter, 1: two-level (8 groups + top), 2: two-level + scalar polls
  float* part;             // split-tile partial slots [max_tiles][2][M][16*nt] f32
  int part_floats;
  unsigned* tickets;       // [max_tiles] zero-initialised, self-resetting
  int max_tiles;
  unsigned long long* ts;  // optional [grid][32] s_memrealtime stamps per workgroup (profiling)
  // optional decode-attention phase in front of the GEMM phases (head_dim 128, attn_g = GQA
  // group size; 0: none): the o_proj weights stream while the attention runs
  DecodeAttnParams attn;
  int attn_g;
  // LDS item (attention launches, M = 1): byte offset of the LDS region that receives phase 1's
  // weight item 2 of every workgroup by LDS-DMA during the attention window (0: off)
  int lds_item;   // (phase 1)
  int lds_item_waves;  // waves whose item 2 is in LDS (the region holds 16 KB per wave)
  int lds_item_req;  // host request for the LDS item (vwa_chain_prepare decides lds_item)
  // LDS item of phase 2 (the down projection, Llama tail): item 2 of every workgroup's range,
  // LDS-DMA'd at the gate/up -> down barrier into the region above phase 2's X rows and
  // reduction scratch; the staging wave (xdma) takes none (0: off)
  int lds_item2;
  int lds_item2_waves;
  int lds_item2_req;  // host request
  // attention -> o_proj hand-off without a grid barrier: every (row group, kv head) final output
  // adds 1 to a counter (bar u64 word 176, reset after the next barrier); only the workgroups
  // with o_proj units wait for the count
  int attn_flag;
  int pre_mask;  // bit i: two weight items issued ahead of the barrier before phase i (xdma issues one)
  int pre_waves;  // > 0: only waves below it issue the next phase's items at a barrier (0: all)
  int xfirst;     // the staging wave's X pieces enter the CU's memory queue before the others' next items
  int xwait;      // no wave issues weights between a barrier's release and its X rows landing in LDS
  int xw_late;    // (xwait) the weights go out after the row scales, not before
  int poll_free;  // wave 0 (the barrier poller) issues nothing ahead of a barrier wait
  int o_nt2;      // attention launches: phase 0 (o_proj) in 32-column tiles (host request; prepare clears it when unused)
  int d_nt2;      // 5..16 rows: the X-streaming down projection in 32-column tiles (host request; cleared when unused)
  int kv_prefetch;  // multi-layer launch: attention workgroups pull their next item's old K/V into L2 while they wait
  int qkv_flags;    // multi-layer launch: QKV -> next attention by per-kv-group tile counters (0: grid barrier)
  int attn_pre;     // attention workgroups (no o_proj units) issue gate/up's item 0 during their attention
  ChainTP tp;
};

// LDS-tiled MFMA GEMM (gemm.hip) for M > 16 rows: Y = epi(rstd[m] * X . W^T (+bias) ...)
struct GemmParams {
  const uint16_t* X; int ldx;       // [M, K] bf16 row-major
  const uint16_t* W; int w_tiled;   // [N, K] bf16: pre-tiled (ops.tile_weight) or row-major
  int M, N, K;
  void* Y; int ldy; int y_f32;      // [M, N] (SwiGLU: [M, N/2]) bf16 or f32
  const uint16_t* bias;             // [N] or null
  const uint16_t* R; int ldr;       // residual (epilogue 1), may alias Y
  const float* rstd;                // [M] per-row scale (RMSNorm with gamma folded into W) or null
  float* ws; int splits; int kg_per_split;  // split-K f32 slabs [splits][M][N] (launcher fills kg_per_split)
  // W8A8 (sw != null): X is OCP e4m3 bytes [M, ldx] with per-row scales sx, W the fp8 tiled layout
  // (ops.tile_weight_fp8) with per-row scales sw
  const float* sx; const float* sw;
  // batched launch (nbatch > 1, no split-K): batch z reads X + z*bsx, writes Y + z*bsy and reads
  // R + z*bsr (element strides; bsr 0 = one residual for every batch, e.g. a positional table).
  // X rows may overlap (ldx < K: the Whisper conv stem as an implicit GEMM, row t = the 3 input
  // rows t*stride-1 .. t*stride+1 of a zero-padded channels-last buffer)
  int nbatch; int64_t bsx, bsy, bsr;
  int cus; int64_t ws_cap;  // CU count and workspace floats (split-K choice of the 256^2 kernel)
  // epilogue 5 (QKV): rotary embedding + paged-KV write of a QKV projection with permuted head rows
  // (ops.permute_qkv_rows: each 16-column tile holds the rotation pairs (c, c + 8)) -- q heads go
  // to q_out in natural dim order, k / v heads to the caches at slots[m] (< 0: not written);
  // Y is not written.  No separate rope_kv_write launch.
  int n_q_heads, n_kv_heads, head_dim, use_rope;
  const int* positions; const int64_t* slots; const float* rope;
  uint16_t* q_out; int ldq; uint16_t* k_cache; uint16_t* v_cache; int block_size;
  int64_t cache_sb, cache_sh, cache_st;
  // RMS statistics hand-off (decode steps of > 16 rows, one rank): ss_out -- the residual epilogue
  // adds the squares of its bf16 output rows into ss_out[m] (the next RMSNorm's statistics);
  // ss_zero[0, ss_zero_n) is zeroed by workgroup 0 (the other buffer, already consumed); ss_in --
  // the per-row scale is rsqrt(ss_in[m] / K + ss_eps) instead of rstd[m] (no row_rstd launch).
  // The sums are u64 fixed point in units of 2^-24 (kSsScale): integer atomics add in any order
  // to the same bits, so the statistics -- and every token after them -- are run-to-run
  // reproducible (f32 atomics were not: tools/repro_check.py)
  unsigned long long* ss_out; unsigned long long* ss_zero; int ss_zero_n; const unsigned long long* ss_in;
  float ss_eps;
};

struct FlashAttnParams {
  const uint16_t* q; int64_t q_stride_b, q_stride_s, q_stride_h;   // q[b][s][h][d]
  KVView kv;                        // keys of sequence b: table row b
  uint16_t* o; int64_t o_stride_b, o_stride_s, o_stride_h;
  int B, Sq, Sk, n_q_heads, n_kv_heads, head_dim;
  int causal;
  int q_offset;                     // absolute position of query 0 (causal: key j visible iff j <= q_offset+i)
  const int* q_offsets;             // optional per-batch q offsets
  const int* k_lens;                // optional per-batch key counts
  float scale;
};

// Persistent Whisper decoder step (whisper_dec.hip wdec_kernel): ONE launch runs every decoder
// layer of a one-row decode step -- seven dependent levels per layer (self-attention QKV, self-
// attention, out-proj + cross-query pre-activation, cross-attention, cross out-proj, fc1, fc2) plus
// one off the critical path (the layer input's share of the cross query), with each workgroup's
// share of a layer's weights held in registers from the previous layer on.
enum { kWdLevels = 8, kWdGemms = 7, kWdRole = 32 };
struct WdecGemm {
  const uint16_t* W;      // pre-tiled bf16 [N / 16][K / 128][4 KB] (ops.tile_weight)
  const uint16_t* bias;   // [N] or null
  const float* ln_c;      // folded LayerNorm column sums [N] (ops.fold_layernorm) or null
};
struct WdecLayer {
  // qkv, out-proj, cross query (LayerNorm gamma folded; bias = its product with the out-proj bias,
  // ln_c = its column sums), cross out-proj, fc1, fc2, cross query x out-proj (bias = the folded
  // cross-query bias, applied after the LayerNorm)
  WdecGemm g[kWdGemms];
  uint16_t* k_cache; uint16_t* v_cache;    // self-attention cache [blocks][H][block_size][64]
  const uint16_t* xk; const uint16_t* xv;  // cross-attention K / V [sessions][T][H][64]
};
struct WdecParams {
  const WdecLayer* layers; int n_layers;
  const int* roles;                   // [grid][kWdRole] (models/whisper.py wdec_roles)
  int d, H, ffn, T, block_size, bt_stride, nch, ch_len, sessions;
  float eps, scale;
  uint16_t* x0; uint16_t* x1;         // hidden row ping-pong (x0: the embedding; result in x[n_layers & 1])
  uint16_t* q; uint16_t* att; uint16_t* f;
  float* xpart;                       // cross-attention partials [H][nch][4 + 64] (max, sum, -, -, out)
  const int* seq_ids; const int* ctx_lens; const int64_t* slots; const int* block_table; const int* cross_table;
  unsigned long long* cnt;            // uncached: level counters [8 levels][8 groups] at 128-byte stride, err word at [1024]
  int n_prod[kWdLevels];              // workgroups that complete each level (per layer)
  unsigned long long* ts;             // diagnostic stamps [grid][n_layers * 8][4] (tools/wdec_probe.py) or null
  int opt[4];                         // schedule options (whisper_dec.hip kOpt*)
  // optional LM head after the last layer (lm_W null: none): folded final LayerNorm, pre-tiled
  // [n_vocab][d] bf16, bias [n_vocab], column sums [n_vocab] -> f32 logits row [n_vocab]
  const uint16_t* lm_W; const uint16_t* lm_b; const float* lm_c; float* logits; int n_vocab;
  // optional: the step's embedding from the tables (tok_emb null: x0 holds it already) -- row
  // tokens[0] of tok_emb [emb_rows][d] (ids outside give zeros) + row positions[0] of pos_emb
  const uint16_t* tok_emb; const uint16_t* pos_emb; const int* tokens; const int* positions; int emb_rows;
  // optional (needs the LM head): greedy masked argmax of the logits (smp_mask: one bit per token,
  // the sampler's; -1 when no token is admissible) and the device-loop advance (asr/engine.py):
  // token -> smp_tok, loop_out[loop_cnt++], adv_tokens[0]; position / context / KV slot move on
  const uint32_t* smp_mask; int* smp_tok; int* smp_step; float* smp_part; int* loop_out; int* loop_cnt;
  int loop_max, loop_base_block;
  int* adv_tokens; int* adv_positions; int* adv_ctx; int64_t* adv_slots;
};

#ifdef __cplusplus
extern "C" {
#endif
int vwa_skinny_gemm(int epi, const SkinnyParams* p, hipStream_t st);
int vwa_skinny_stream(int epi, const SkinnyParams* p, int grid_cap, int ks, hipStream_t st);
void vwa_skinny_set_x_skew(int skew);  // LDS-staged X rows: 64-B skew every 4 rows (default) or none (0)
int vwa_chain_prepare(ChainParams* cp, int grid);
// n_layers > 1: d_cp is an array of n_layers descriptors of consecutive 4-phase Llama tails with the
// attention phase, run by ONE launch (skinny_stream.hip chain_kernel MULTI)
int vwa_chain_launch(const ChainParams* d_cp, int seq, int n_phases, int attn_g, int lds, int grid, hipStream_t st,
                     int xg2 = 0, int f8 = 0, int o2 = 0, int n_layers = 1);
// -10: a shape / role table the kernel does not take (the caller keeps per-kernel launches)
int vwa_wdec_launch(const WdecParams* p, int grid, hipStream_t st);
int vwa_gemm(int epi, const GemmParams* p, hipStream_t st);
int vwa_gemm_splits(int M, int N, int K, int cus, int64_t ws_floats, int f8);
void vwa_gemm_set_split_fill(int pct);  // split-K while tiles x splits < pct % of the CUs (0: bf16 75, fp8 100)
void vwa_gemm_set_p8(int mode);  // 0: 128^2 kernel only, 1: 256^2 8-phase wherever eligible, 2: measured rule
int vwa_row_rstd(const uint16_t* x, int ldx, int M, int K, float eps, float* rstd, hipStream_t st);
int vwa_rmsnorm(const uint16_t* x, const uint16_t* residual, uint16_t* residual_out, const uint16_t* w,
                uint16_t* y, int rows, int D, int ldx, float eps, hipStream_t st);
int vwa_layernorm(const uint16_t* x, const uint16_t* residual, uint16_t* residual_out, const uint16_t* w,
                  const uint16_t* b, uint16_t* y, int rows, int D, int ldx, float eps, hipStream_t st);
int vwa_rope_kv_write(const uint16_t* qkv, int ldqkv, int rows, int n_q_heads, int n_kv_heads, int head_dim,
                      int use_rope, const int* positions, const int64_t* slots, const float* rope, uint16_t* q_out,
                      int ldq, uint16_t* k_cache, uint16_t* v_cache, int block_size, int64_t sb, int64_t sh,
                      int64_t st_, hipStream_t st);
int vwa_swiglu(const uint16_t* gu, uint16_t* h, int rows, int F, hipStream_t st);
int vwa_bias_act(const uint16_t* x, const uint16_t* bias, const uint16_t* residual, uint16_t* y, int rows, int N,
                 int act, hipStream_t st);
int vwa_decode_attention(const DecodeAttnParams* p, hipStream_t st);
void vwa_set_attention_impl(int impl);  // 1: multi-query MFMA kernel (default), 0: split VALU kernel
int vwa_flash_attention(const FlashAttnParams* p, hipStream_t st);
int vwa_embedding(const int* ids, const uint16_t* table, const uint16_t* pos_table, const int* positions,
                  uint16_t* out, int rows, int D, int vocab_start, int vocab_end, hipStream_t st);
int vwa_sample(const float* logits, int ld, int rows, int V, const uint32_t* mask, int mask_words,
               const float* temperature, const uint64_t* seed, const int* step, int* out_tokens,
               float* part_val, int* part_idx, int n_chunks, const int64_t* fail_word, hipStream_t st);
// vocab-parallel sampling stages: partial maxima over the local vocab shard (global token ids =
// v_off + local column; mask rows indexed by global id), then the merge of n_src ranks' partials
// (rank p's at part_val / part_idx + p * src_stride)
int vwa_sample_partial(const float* logits, int ld, int rows, int V, int v_off, const uint32_t* mask, int mask_words,
                       const float* temperature, const uint64_t* seed, const int* step, float* part_val,
                       int* part_idx, int n_chunks, hipStream_t st);
int vwa_sample_final(const float* part_val, const int* part_idx, int n_chunks, int n_src, int64_t src_stride,
                     int* out_tokens, int* step, int rows, const int64_t* fail_word, hipStream_t st);
int vwa_pcm16_to_f32(const int16_t* pcm, float* out, int n_in, int n_out, float ratio, hipStream_t st);
// basis: DFT cos/sin fragments [26 tiles][25][64][4] f32, fb_frag: mel filterbank fragments
// [n_mels/16][13][64][4] f32 (ops.logmel_tables)
int vwa_log_mel(const float* audio, int n_samples, int n_frames, const float* window, const float* basis,
                const float* fb_frag, int n_mels, float* mel_out, float* max_buf, uint16_t* out_bf16, int ld_out,
                hipStream_t st);
int vwa_attention_split_tokens();
int vwa_decode_advance(int* tokens, int* positions, int* ctx_lens, int64_t* slots, const int* sampled,
                       int* out, int* counter, int max_out, int base_block, int block_size, hipStream_t st);
int vwa_quant_fp8_rows(const uint16_t* x, int ldx, int rows, int D, uint8_t* q, float* scale, float* rstd, float eps,
                       hipStream_t st);
// one-shot peer-to-peer all-reduce (allreduce.hip)
void* vwa_ar_create(int rank, int world, int64_t max_elems);
int vwa_ar_handles(void* st, void* out);
int vwa_ar_handle_bytes();
int vwa_ar_open_peer(void* st, int p, const void* in);
int vwa_ar_allreduce(void* st, const uint16_t* in, uint16_t* out, int64_t n, hipStream_t stream);
int vwa_ar_gather(void* st, const int* in, int* out, int64_t n, hipStream_t stream);
int64_t vwa_ar_gather_max_words();
int vwa_ar_chain_tp(void* st, ChainTP* out);
int vwa_ar_error(void* st);
void vwa_ar_destroy(void* st);
#ifdef __cplusplus
}
#endif
