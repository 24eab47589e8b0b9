// fw_internal.h — shared device/host definitions of the MI355X window operator.
//
// HBM layout of the keyed state ("window-contents" + event-time timers):
//   The KeyGroupRange owned by a handle is split into P = nKG << logS state partitions
//   (a key group keeps its partitions contiguous, so a per-key-group snapshot is a contiguous
//   slice — HeapKeyedStateBackend.java:370-381 writes state per key group the same way).
//   Partition p owns a region of R = 1 << logR open-addressing slots in each of two table
//   buffers; cur[p] says which buffer is live.  A slot is a 64-byte Entry (one cache line:
//   key, window start/end, the accumulator and timer flags) plus a 4-byte state word kept in
//   a separate dense array so an empty region is cleared with a contiguous 4R-byte memset.
//   The event-time timers of HeapInternalTimerService (HeapInternalTimerService.java:224-290)
//   are not materialised: an entry's trigger timer is the FW_TIMER flag (set when an element
//   is added while maxTimestamp > watermark, EventTimeTrigger.java:37-45; cleared when it
//   fires) and its GC timer is implied by the entry's existence (cleanupTime,
//   WindowOperator.java:637-644).  next_timer[p] is the earliest timer in region p, so a
//   watermark only visits regions that have something to fire or clean.
#pragma once
#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifndef FW_TILE
#define FW_TILE 16384          // records per classify/scatter workgroup (with FW_RPT 4 against 32768 / 8: C2 +2.6 %, C4 +2.8 %, C1 +1 %, C3 -2.4 %, C5 / C5t even)
#endif
#ifndef FW_TILE_THREADS
#define FW_TILE_THREADS 1024   // classify / scatter workgroup
#endif
#ifndef FW_RPT
#define FW_RPT 4               // records per thread kept in flight by the streaming kernels (even: pairs)
#endif
#ifndef FW_XCD_TILES
#define FW_XCD_TILES 0         // 1: consecutive tiles of a partition's run on one XCD (blocks b, b+8, ...)
#endif
#ifndef FW_AGG_RPT
#define FW_AGG_RPT 2           // the same for k_aggregate: 2 keeps it at 80 VGPRs = 3 workgroups per CU
#endif
// minimum waves per SIMD the compiler must leave room for (register budget); 1 = no constraint
#ifndef FW_AGG_WAVES
#define FW_AGG_WAVES 6  // 80 VGPRs: 3 workgroups of 512 per CU (86 unconstrained gave 2; measured 0.425 -> 0.371 ms at C2)
#endif
#ifndef FW_GATHER_WAVES
#define FW_GATHER_WAVES 4  // the gathered instantiation: its runs table takes 12 KB of LDS, 2 workgroups per CU
#endif
#ifndef FW_POOL_RPT
#define FW_POOL_RPT FW_AGG_RPT  // the same for the pooled (HyperLogLog, t-digest) one-window instantiation
#endif
#ifndef FW_PLAIN_RPT
#define FW_PLAIN_RPT FW_AGG_RPT  // ... and the plain count/sum/min/max one (not the dense regions)
#endif
#ifndef FW_SESS_RPT
#define FW_SESS_RPT 1  // records per thread in flight in the count/sum/min/max session instantiation (1: 1.19e10 -> 1.24e10 at C4 against 2; 3, 4 slower)
#endif
#ifndef FW_SESS_WAVES
#define FW_SESS_WAVES 4  // the same for the session instantiation
#endif
#ifndef FW_SCATTER_WAVES
#define FW_SCATTER_WAVES 1
#endif
#define FW_AGG_THREADS 512     // aggregate workgroup
#ifndef FW_AGG_CHUNK
#define FW_AGG_CHUNK 32768     // records per aggregate workgroup of a split partition (hot keys); 16384 -> 32768: C4 6.9e9 -> 7.7e9, C5 6.1e9 -> 6.7e9 records/s
#endif
#ifndef FW_HLL_AGG_CHUNK_MUL
#define FW_HLL_AGG_CHUNK_MUL 2  // HyperLogLog over time windows: FW_AGG_CHUNK times this per split workgroup
#endif
#ifndef FW_LDS_SLOTS
#define FW_LDS_SLOTS 1024      // LDS pre-aggregation slots per aggregate workgroup (a power of two)
#endif
#ifndef FW_LDS_FILL_LIMIT
#define FW_LDS_FILL_LIMIT 820  // ~0.8 * FW_LDS_SLOTS: a new slot is not claimed beyond this fill
#endif
#define FW_FIRE_THREADS 256
#ifndef FW_TD_T1
#define FW_TD_T1 128           // t-digest: digests with at most this many batch values + centroids merge serially (16 / 32 / 64 / 128 / 256 / 512: C5t 3.68 / 3.92 / 4.10 / 4.18 / 4.11 / 3.93e9)
#endif
#ifndef FW_TD_T3
#define FW_TD_T3 2048          // ... at most this many in one wave; more over the whole grid (the hottest keys)
#endif
#define FW_SLOW_THREADS 1024
// Dense tumbling regions (DevCfg::dense): the LDS table of k_dt_aggregate (slots, threads, records per thread in
// flight).  Regions are sized for about FW_DT_SLOTS * 3/4 live entries each.
#ifndef FW_DT_SLOTS
#define FW_DT_SLOTS 2688
#endif
#ifndef FW_DT_THREADS
#define FW_DT_THREADS 1024
#endif
#ifndef FW_DT_RPT
#define FW_DT_RPT 2
#endif
#ifndef FW_DT_NDEPTH
#define FW_DT_NDEPTH 2  // narrow records: rounds of raw pairs in flight (0: two widened rounds, as 16-byte records)
#endif
// Tile-local ("gathered") partitioning of compact count/sum/min/max batches: k_stage sorts each tile of
// FW_GTILE records by partition in LDS and writes it back linearly (a wave's stores are whole lines; scattered
// 16-byte stores into partition-major runs measured 2.4x slower), and k_aggregate gathers a partition's runs
// from every tile through the runs table.  P <= FW_GMAX_P (the staging's LDS) and at most FW_GMAX_T tiles per
// batch (the aggregate's LDS copy of a partition's row of the runs table).
#define FW_GTILE 8192
#define FW_GMAX_P 2048
#define FW_STAGED_MAX_P 4096  // LDS-staged offset scatter (k_scatter_staged): up to this many partitions
#define FW_GMAX_T 2048
#define FW_REGROUP_THREADS 512
#define FW_REGROUP_CHUNK 16384  // records per regroup workgroup (a hot partition takes several)
// DIAG_AGG_TIMING's clocks and printf are compiled in only on request: the printf calls cost k_aggregate
// its registers (a call saves the live VGPRs to scratch)
#ifndef FW_AGG_TIMING_BUILD
#define FW_AGG_TIMING_BUILD 0
#endif

enum : uint32_t { SLOT_EMPTY = 0, SLOT_LIVE = 1, SLOT_DEAD = 2, SLOT_BUSY = 3 };
enum : int64_t { FW_TIMER = 1 };

struct TdCent;
struct DevCfg {
  int32_t assigner, vtype, key_kind, purging;
  int32_t side_output, max_par, kg0, n_kg;
  int32_t log_s, P, log_r, wpr;  // wpr = max windows per record
  int64_t size, slide, offset, gap, lateness;
  int32_t diag;                  // FW_DIAG ablation bits (diagnostic builds of the timing only; 0 in production)
  // the field's width (FW_VAL_I16 / I8 / F32 are kept as I32 / F64 inside): sums wrap to sum_bits (64, 32, 16
  // or 8) and a Float field's sum is rounded to float, when rows and snapshots are written
  int32_t sum_bits, f32;
  // sliding windows as panes (size % slide == 0, allowedLateness 0): the state holds one entry per
  // (key, pane) = (key, [p, p + slide)), and a window [s, s + size) is the merge of its size/slide
  // panes, formed when it fires.  An entry's meta is then the end - 1 of the earliest window it has
  // not yet been fired into (its timer); nt_floor = the earliest window end after the launch's
  // watermark (set per launch by the host).
  int32_t panes;
  int64_t nt_floor;
  // Block pool of the user AggregateFunctions whose accumulator does not fit an Entry: one block of
  // pool_bytes per live (key, window), the entry's block id is meta >> 1.  Free blocks are kept on a
  // stack: pool_ctr[0] = stack height, pool_ctr[1] = blocks ever handed out from the end of the pool.
  //   FW_AGG_HLL: 2^hll_p one-byte registers (zeroed when freed).
  //   FW_AGG_TDIGEST: TdHead + two halves of td_nb centroids (TdCent); the live half is TdHead::cur.
  int32_t agg, hll_p;
  // FW_AGG_FIRST: arrival ordinal of record 0 of the launch's batch (set per push by the host).  The
  // entry's mx holds ~ordinal of the window's first element, so the max merges everywhere keep it.
  int64_t ord_base;
  int64_t* slow_ord;  // [max_batch] ordinal of each ordered-path record (the push's scratch set)
  const int64_t* by_val;  // FW_AGG_MINBY / MAXBY: the batch's value column by batch index (the push's scratch set)
  uint8_t* pool;
  uint32_t* pool_free;
  int32_t* pool_ctr;      // [0] stack height, [1] blocks handed out from the pool's end, [2] deferred frees
  // blocks freed by a session merge while the aggregate or the ordered path may pop others (already zeroed):
  // pushed on the free stack by the next firing (k_pool_release), when nothing pops
  uint32_t* pool_defer;
  // t-digest over session windows (merging): the session merges of a push, logged by the session flush and the
  // ordered replay (target block, merged block; td_mctr[0] entries), and the ordered path's added elements (key,
  // timestamp, value; td_ovctr[0]) for the compression at the end of the push
  uint32_t *td_mdst, *td_msrc;
  int32_t* td_mctr;
  int64_t *td_ovk, *td_ovt, *td_ovv;
  int32_t *td_ovp, *td_ovctr;  // (the added element's state partition)
  // t-digest under allowed lateness (tumbling / sliding): an ordered-path element's td_ovt is its newest window's
  // start and td_ovn its count of non-late windows (the newest ones); a window that fires late compresses its
  // centroids with the push's values so far (td_olast[state slot] -> td_olink[element * wpr + window] chain)
  // into its thread's td_late scratch (FW_SLOW_THREADS x td_nb)
  int32_t *td_ovn, *td_olast, *td_olink;
  TdCent* td_late;
  // ... and session windows under allowed lateness: the blocks merged into a block during the push (td_bhead[block]
  // -> td_bnext chain), and a late firing's union of their centroids in its thread's td_lateu scratch
  // (FW_SLOW_THREADS x td_lateu_cap)
  int32_t *td_bhead, *td_bnext;
  TdCent* td_lateu;
  int32_t td_lateu_cap;
  int64_t pool_blocks;
  int64_t pool_bytes;     // 0 = no pool
  // FW_AGG_TDIGEST (definition: oracle/window_oracle.h OR_AGG_TDIGEST): td_nb = delta / 2 buckets of the
  // k1 scale function, td_qb[0 .. td_nb] their bounds sin(pi b / delta)^2 (device), quantiles of the rows
  int32_t td_nb;
  const double* td_qb;
  double td_quant[3];
  // invariant-divisor reciprocals (Granlund-Montgomery round-up method) for `% size` / `% slide`
  uint64_t mag_size, mag_slide;
  int32_t l_size, l_slide;
  // sessions: keys that have an ordered-path record in the current batch ("tainted": all their records
  // of the batch are replayed in arrival order).  Open addressing; a slot belongs to the batch whose
  // epoch it holds, so the set is never cleared.
  uint64_t* taint_key;
  uint32_t* taint_state;
  uint32_t taint_mask, taint_epoch;
  // the push's input columns are 16-byte aligned (key_hash 8-byte): the streaming kernels load two
  // consecutive records per lane with 16-byte loads (8-byte lane loads run at ~0.6x the 16-byte rate)
  int32_t vec_in;
  // compact partitioned records (CRec, 16 B instead of PRec's 32 B) for one-window records (tumbling,
  // panes) of the order-free aggregates: the key is kept as fmix64(key ^ SUB_SALT), whose top log_s bits
  // are the record's sub-partition (known to the partition's workgroup), so those bits carry the window
  // instead: d = (start - cbase) / slide in [0, 2^log_s).  `compact` = the configuration allows it (set at
  // creation; 0 for this launch when the watermark gives no representable base); a batch with a normal
  // record whose window is out of range sets *DevCfg::wide and goes through PRec.
  int32_t compact;
  int64_t cbase;
  // the batch's "some record has no compact form" flag (set by k_classify_hist, read by the kernels that read
  // its partitioned records); one word per scratch set, so the next batch's classify may run beside them
  int32_t* wide;
  // dense regions (tumbling windows, count/sum/min/max, allowed lateness 0): a region's live entries sit in slots
  // [0, live) of its current buffer, without state words; k_dt_aggregate rewrites a region into its other buffer
  // from an LDS table, k_dt_fire streams it (fw_device.hip, "dense tumbling regions")
  int32_t dense;
  int32_t agg_chunk;  // records per aggregate workgroup of a split partition (FW_AGG_CHUNK, or twice it)
  // narrow records (round 6; dense single-pass batches of an integer field): the single pass writes 8 bytes per
  // record, {key (29-bit signed) | window delta - ndn0 (3 bits) | value (int32)}, when every record of the batch has
  // that form; a record without it sends the batch through classify / scan / offset scatter (16-byte CRec) and the
  // operator stops trying (fw_runtime.cpp).  Set per launch: 1 = the single pass writes narrow records.
  int32_t narrow;
  int32_t ndn0;       // the window delta (compact_delta) of narrow window 0: the watermark's window
  // FW_AGG_ROW (Table API group windows, oracle/window_oracle.h OR_AGG_ROW): row_nc value columns of FW_VAL_* types,
  // row_ns aggregates (FW_ROW_* << 8 | column).  A window's block holds one RowAcc per column; a record's value is
  // its batch index, and its columns are read from the push's copy: column j of record i at row_cols[j * row_stride
  // + i], its null mask at row_nulls[i] (bit j = column j is NULL; nullptr = none)
  int32_t row_nc, row_ns;
  const int32_t* row_ts;  // [24] in HBM: the columns' types (8), then the aggregates (16) (kept out of DevCfg: a
                          // kernel that changes its DevCfg copy holds it in registers and scratch)
  const int64_t* row_cols;
  const uint8_t* row_nulls;
  int64_t row_stride;
};
// FW_AGG_ROW accumulator of one column (40 bytes, zero = empty): the non-null count, the sum (integral columns: 128
// bits, two's complement, lo / hi; floating columns: f64 in lo), min / max as order keys encoded so that 0 is the
// identity of an unsigned max (row_enc_min / row_enc_max)
struct RowAcc {
  unsigned long long nn, lo;
  long long hi;
  unsigned long long mn, mx;
};

// host: reciprocal of d >= 1 for div_inv(): m = floor(2^64 (2^l - d) / d) + 1, l = ceil(log2 d)
inline void make_div_inv(uint64_t d, uint64_t* m, int32_t* l) {
  int32_t L = 0;
  while (L < 64 && (1ull << L) < d) L++;
  const unsigned __int128 two_l = (unsigned __int128)1 << L;
  *m = (uint64_t)((((unsigned __int128)1 << 64) * (two_l - d)) / d + 1);
  *l = L;
}
// FW_DIAG bits: results are WRONG when any is set; used only to price one stage of a kernel
enum {
  DIAG_AGG_NO_FLUSH = 1,
  DIAG_AGG_NO_LDS = 2,
  DIAG_SCATTER_NO_STORE = 4,
  DIAG_SCATTER_LINEAR = 8,
  DIAG_AGG_NO_ACCUM = 16,  // LDS lookup/claim only, no accumulate atomics
  DIAG_SCATTER_SINGLE = 128, // k_scatter: each lane stores its own record (no lane-pair sectors)
  DIAG_AGG_TIMING = 256,     // k_aggregate prints per-workgroup phase clocks (builds with FW_AGG_TIMING_BUILD=1)
  DIAG_SCATTER_HALF = 512,   // k_scatter stores 16 B per record (the timing of a compact record)
  DIAG_SCATTER_NT = 1024,    // k_scatter stores with nontemporal stores
  DIAG_DT_WIDE = 2048        // k_dt_aggregate: the wide LDS table for every region (timing of the compact table)
};

struct __attribute__((aligned(64))) Entry {
  int64_t key, start, end, cnt, sum, mn, mx, meta;
};

// a record in its partition's run: one 32-byte sector per record, so the scatter writes whole
// sectors (three 8-byte columns scattered separately cost ~4x the bytes in partial writes).
// The window assignment is done once, by the scatter: `last` is the newest window's start and
// `nwin` the number of windows (1 for tumbling), newest first as SlidingEventTimeWindows emits them.
struct __attribute__((aligned(32))) PRec {
  int64_t key, last, val, nwin;
};
// compact form (DevCfg::compact): {fmix64(key ^ SUB_SALT) with the window delta in its top log_s bits, val}
struct __attribute__((aligned(16))) CRec {
  int64_t kw, val;
};

// FW_AGG_HLL register block: a bitmap of the block's 16-byte register chunks that hold a nonzero register
// (set when a register first leaves zero), then the 2^p registers.  The fire reads and zeroes only the marked
// chunks: a window of a few hundred items touches a few hundred of the 2^p / 16 chunks.
__host__ __device__ inline int64_t hll_hdr_bytes(int p) {
  int64_t b = ((int64_t)1 << p) / 128;  // one bit per 16-byte chunk
  if (b < 16) b = 16;
  return (b + 15) & ~(int64_t)15;
}

// region state word: kind in bits 0-1, 24-bit fingerprint of the slot hash in bits 8-31, so a
// probe rejects most foreign slots without reading the 64-byte entry
__host__ __device__ inline uint32_t st_kind(uint32_t s) { return s & 3u; }

struct Status {
  unsigned long long out_rows;        // rows written to the output buffer (monotonic until reset)
  unsigned long long side_rows;       // rows written to the side buffer (monotonic until reset)
  unsigned long long late_dropped;    // numLateRecordsDropped
  unsigned long long fired_total;
  unsigned long long slow_total;
  unsigned long long merged;          // LDS deltas merged into HBM regions (k_aggregate)
  unsigned long long td_cent;         // FW_AGG_TDIGEST: centroids of the fired digests
  unsigned long long partial_records; // records inside the partials pushed (fw_push_partials_device): numRecordsIn
  long long slow_resume;              // ordered path: first list index not yet replayed
  long long need_out;                 // fired-row capacity the ordered path asked for when it suspended
  int32_t need_live;                  // largest live count a region asked for when it suspended
  int32_t flags;                      // FW_STATUS_*
  int32_t kg_errors;
  int32_t ts_errors;
  int32_t suspended;                  // FW_SUSP_*: later kernels of the push / watermark skip themselves
  int32_t need_grow;                  // some region is over half full: grow before it has to suspend
  int32_t taint_any;                  // sessions: 0 no tainted key in the batch, 1 check the set, 2 set full: all
  int32_t rsv_fallbacks;              // single-pass batches that had to go through classify / scan / scatter
  int32_t acc_refused;                // restore: t-digest rows of a window already present, malformed digests
  int32_t narrow_misses;              // narrow single-pass batches redone because a record had no narrow form
};
enum {
  FW_STATUS_STATE_LOST = 1,  // a window could not be stored (more in-flight sessions of one key than supported)
  FW_STATUS_OUT_FULL = 2,
  FW_STATUS_MERGE_LATE = 4,
  FW_STATUS_SIDE_FULL = 8,
  FW_STATUS_POOL = 16,       // the accumulator block pool (HyperLogLog registers, t-digests) ran out of blocks
  FW_STATUS_TD_UNION = 32    // a late session firing joined more centroids than its union scratch holds
};
// a region takes new windows only up to this load; beyond it the kernel suspends and the table grows
__host__ __device__ inline int32_t region_limit(int32_t log_r) { return (int32_t)((3ll << log_r) >> 2); }
// suspension: a kernel stopped before changing anything it cannot keep (a region or the fired-row
// buffer lacked room); the host grows the table / buffer and resumes exactly where it stopped
enum { FW_SUSP_AGG = 1, FW_SUSP_SLOW = 2, FW_SUSP_FIRE = 4 };

// k_aggregate progress, kept per partition so a suspended launch can be resumed
struct AggProg {
  long long* rb;     // [P] first record of the round to restart from
  uint32_t* tp;      // [P * FW_AGG_THREADS] per thread: record (bits 0-7), window (bits 8-31) in that round
  uint8_t* done;     // [P] partition finished in this push
};

// Partitions longer than FW_AGG_CHUNK records (hot keys) are split: one k_aggregate workgroup per
// chunk pre-aggregates its records in LDS and writes the LDS entries as deltas (Entry form) at the
// chunk's own record indices; the last chunk of the partition to finish merges all the deltas into
// the region.  Tumbling windows and sessions only (one delta per record at most).
struct AggHot {
  Entry* delta;          // [max_batch]
  uint32_t* chunk_base;  // [P + 1] exclusive scan of the chunks per partition; nullptr = no splitting
  uint32_t* scan_tmp;
  int32_t* nd;           // [chunks] deltas written by each chunk
  uint32_t* pdone;       // [P] chunks of the partition finished
};

struct DevTable {
  Entry* ent[2];
  uint32_t* state[2];
  uint8_t* cur;
  int32_t* live;
  int64_t* next_timer;
  int64_t* fire_e;     // panes: window maxTimestamp a suspended k_fire resumes at, LMIN = from the start
  uint64_t* fire_lo;   // panes: first key hash of that window not yet emitted
  int64_t* pane_floor; // panes: every window of the region with maxTimestamp < pane_floor has been formed
  uint8_t* passes;     // dense regions: log2 of the hash passes the region's last aggregate needed (a hint)
};

struct DevRows {
  int64_t *key, *start, *end, *cnt, *sum, *mn, *mx;
  int64_t* dig;        // FW_AGG_TDIGEST with export: per row [n, (sum bits, weight) x td_nb] (nullptr = off)
  int64_t cap;
  int64_t slow_limit;  // the ordered path stops here, leaving room for one watermark's firing (cap - table slots)
};
// ---- t-digest blocks (FW_AGG_TDIGEST): a 16-byte head, then two halves of td_nb centroids each
struct TdHead {
  int32_t cur;    // live half
  int32_t n;      // centroids in it
  int64_t w;      // their total weight (elements compressed so far)
};
struct TdCent {
  double sum;     // the centroid's elements added left to right (mean = sum / weight)
  int64_t cum;    // total weight of this and every earlier centroid
};
// per-push buffers of the t-digest compression (fw_runtime.cpp allocates them for max_batch records)
struct TdLarge {  // a digest whose batch is compressed bucket-parallel
  int64_t beg, nn;          // its values in the sorted batch
  int64_t W;                // total weight after the batch
  int32_t no;               // old centroids
  int32_t pad;
  const TdCent* old;        // live half
  TdCent* out;              // the other half (group sums per bucket, then the centroids)
  TdHead* head;
};
struct TdOverride {  // a merged digest's old centroids (instead of its live half) and their total weight
  const TdCent* old;
  int32_t no;
  uint32_t slot;  // the digest's global slot (its mover entry)
  int64_t wold;
};
// the batch's values grouped by digest, then sorted within each digest's run (launch_tdigest): runs sorted in LDS
// (<= TD_SORT_MAX values) and longer runs split first by sample-sort passes
struct TdRun {
  uint32_t beg, len;        // len bit 31: the values are in v[1] (else v[0])
};
struct TdMsd {
  uint32_t toff;            // the run's first tile (TD_TILE values each) among the level's runs
  uint32_t nsp;             // its splitters (td.spl)
};
#define FW_TD_LC_WORDS 21
struct TdBuf {
  uint32_t* gs[2];          // per item: [0] its digest's global slot (partition << log_r | slot), [1] its rank in the run
  uint64_t* v[2];           // per item its Double.compare-ordered value key; [1] the values grouped by digest, [0]
                            // each digest's run sorted (the tiers read v[0])
  uint32_t* binv;           // [pool blocks] global slot of each block's entry (rewritten when it moved)
  uint32_t* dcnt;           // [table slots] a digest's items in the batch, then its run's start (zero between pushes)
  uint32_t* gsort;          // [max items] the digest of each sorted position (`none` past the runs)
  TdRun* lrun;              // [lrun_cap] runs for the LDS sort
  TdRun* brun[3];           // [brun_cap] runs for MSD pass 1, 2, and the fallback
  TdMsd* msd;               // [brun_cap] the sample-sort level's runs' tiles and splitter counts
  uint64_t* spl;            // [brun_cap * 2047] their splitters
  uint32_t* hist;           // [brun_cap * 4096] their buckets' counts, then cursors
  int32_t* lctr;            // [FW_TD_LC_WORDS] [0] lrun entries, [1..3] brun[0..2] entries, [4] the MSD level's
                            // tiles, then the serial tier's length classes (k_td_starts, k_td_perm)
  int64_t lrun_cap, brun_cap;
  uint32_t* tslot;          // touched digests: global slot      [max_batch]
  uint32_t* tbeg;           //                  first sorted value [max_batch]
  int32_t* ctr;             // [0] touched digests, [1] large ones, [2] wave-tier ones
  uint32_t* mid;            // [max_batch] the wave tier's digests (touched indices)
  TdLarge* large;           // [max_large]
  int32_t* nstart;          // [max_large * td_nb] first sorted value of each bucket (-1: none)
  int32_t* ostart;          // [max_large * td_nb] first old centroid of each bucket (-1: none)
  uint64_t* okey;           // [max_large * td_nb] the large digests' old centroids' mean keys
  int32_t* lidx;            // [table slots] large index of a touched digest, -1 = compressed serially
  int64_t lidx_slots;
  int32_t max_large;
  // session merges (DevCfg::td_mdst / td_msrc): a merged digest's old centroids are the union of its own and of the
  // digests merged into it, ordered by (mean, weight, sum), built once per push into `uni`; the tiers read them
  // through the override of the digest's slot
  uint32_t* fwd;            // [pool blocks] the block a block was merged into (~0: none)
  int32_t* mhead;           // [pool blocks] a final target's list of merge-log entries (-1: none)
  int32_t* mnext;           // [pool blocks] next entry of that list (-1: end); -2: the entry that builds the union
  int32_t* mover;           // [table slots] override index of a digest's slot (-1: none)
  TdOverride* ovr;          // [pool blocks]
  TdCent* uni;              // [pool blocks * td_nb] the unions' centroids
  unsigned long long* uctr; // [2]: centroids of `uni` taken, overrides taken
};

// ---- count windows (FW_COUNT): per key its element count and a ring of its last size-1 elements
struct DevCount {
  int64_t* mkey;        // [cap] key map: keys (open addressing)
  uint32_t* mstate;     // [cap] 0 empty, 1 being claimed, 2 taken
  uint32_t* mslot;      // [cap] the key's slot
  int32_t* nslots;      // slots handed out
  int64_t* cnt;         // [max_keys] elements of the key so far (CountTrigger's count, the list's length)
  int64_t* ring_v;      // [max_keys * (wl - 1)] the key's last wl - 1 values, at (seq - 1) % (wl - 1)
  int64_t* ring_o;      //                             and their arrival ordinals
  uint32_t cap_mask;
  int32_t max_keys;
  int64_t size, slide;
  int64_t wl;           // the fired window's length: size (evict before) or size + slide (evict after)
  uint32_t* sk[2];      // per batch: sort keys (slot) / values (batch index), double-buffered for the sort
  uint32_t* sv[2];
  void* tmp;
  size_t tmp_bytes;
  int32_t* sbeg;        // [max_keys] the key's run in the sorted batch
  int32_t* send;
};

// columns of keyed-state snapshot rows (fw_state_rows, device side)
struct StateCols {
  int64_t *key, *start, *end, *cnt, *sum, *mn, *mx, *timer;
  // block-pool aggregates (DevCfg::pool_bytes): a snapshot writes each row's block id into blk; a restore
  // hands blk[(*used)++] to each new (key, window) and imports row i's accumulator from acc + i * acc_bytes
  int64_t* blk;
  const uint8_t* acc;
  int64_t acc_bytes;
  int32_t* used;
};
struct DevSide {
  int64_t *key, *ts, *val;
  int64_t cap;
};
// pre-shuffle combining: partial accumulators of (key, window) in the table's own representation
struct PartialCols {
  int64_t *key, *start, *cnt, *sum, *mn, *mx;
};
struct PartialRec {
  int64_t key, start, cnt, sum, mn, mx;
};

// ---------------------------------------------------------------- launchers (fw_device.hip)
typedef hipStream_t hipStream_t_;
namespace fwdev {
// fw_profile's dispatch timing (set by the runtime around one launch helper): when `a` is set, the helper issues
// its kind's main kernel with hipExtLaunchKernelGGL and these start / stop events, which take that dispatch's own
// timestamps instead of marker packets on the stream, and sets `used`
struct ExtTiming {
  hipEvent_t a, b;
  bool used;
};
extern thread_local ExtTiming g_ext;
void launch_classify_hist(const DevCfg& c, int64_t wm, const int64_t* key, const int64_t* ts, const int32_t* kh,
                          int64_t n, int32_t T, uint32_t* hist, Status* st, hipStream_t_ s,
                          const uint32_t* rsv = nullptr);
// in-place exclusive; gate: the scan runs only when *gate != 0 (nullptr = always)
void launch_scan(uint32_t* data, int64_t m, uint32_t* scratch, hipStream_t_ s, const uint32_t* gate = nullptr);
void launch_scatter(const DevCfg& c, int64_t wm, const int64_t* key, const int64_t* ts, const int64_t* val,
                    const int32_t* kh, int64_t n, int32_t T, uint32_t* offs, PRec* part, int64_t* sk,
                    int64_t* stt, int64_t* sv, int32_t* skh, DevSide side, Status* st, hipStream_t_ s,
                    const uint32_t* gate = nullptr);
// single-pass scatter of a dense compact batch (k_scatter_staged<..., true>): partition p's run at [p * rcap,
// p * rcap + rsv[p]); rsv holds P + FW_RSV_WORDS words, zeroed before the launch.  When rsv[P] is set after it, the
// batch goes through launch_classify_hist / launch_scan / launch_scatter gated on rsv (they do nothing otherwise).
#define FW_RSV_WORDS 8
#define FW_RSV_WIDE 3  // rsv[P + FW_RSV_WIDE]: the batch's DevCfg::wide word when it took the single pass
#define FW_RSV_NARROW 6  // rsv[P + FW_RSV_NARROW]: a narrow single pass met a record without a narrow form
bool rsv_eligible(const DevCfg& c);
// the single-pass words (P + FW_RSV_WORDS) zeroed after the batch's aggregate, unless the push suspended
void launch_rsv_reset(uint32_t* rsv, int32_t words, const Status* st, hipStream_t_ s);
void launch_scatter_rsv(const DevCfg& c, int64_t wm, const int64_t* key, const int64_t* ts, const int64_t* val,
                        const int32_t* kh, int64_t n, int32_t T, PRec* part, uint32_t* rsv, int64_t rcap, hipStream_t_ s);
// hot: chunk splitting of long partitions (nullptr = one workgroup per partition); n = records of the push
// gathered batches (FW_GTILE): offs = the partitions' virtual offsets (P + 1, T = 1), rt_t = the runs table
// [P][T8] (tile-local start | count << 16), t8 = tiles of the batch; rt_t = nullptr for partition-major runs
void launch_aggregate(const DevCfg& c, int64_t wm, const PRec* part, const uint32_t* offs, int32_t T, DevTable tb,
                      AggProg prog, int resume, const AggHot* hot, int64_t n, Status* st, hipStream_t_ s,
                      const uint32_t* rt_t = nullptr, int32_t t8 = 0, const uint32_t* rsv = nullptr,
                      int64_t rcap = 0);
// gathered batches: classify + tile-local partition sort (k_stage, into the second half of part: mb = its
// capacity in PRecs), the runs table's transpose and the partitions' virtual offsets (voffs, P + 1), the
// ordered-path compaction (srow: scanned ordered-path counts per tile, then the raw counts; 2 x t8) and the
// regroup of every partition's runs into compact partition-major runs at the start of part (offsets voffs, T = 1);
// scan_tmp: P + 1 words for the regroup's chunk bases
int gather_mode(const DevCfg& c, int64_t n);  // host: the batch can be gathered
void launch_stage(const DevCfg& c, int64_t wm, const int64_t* key, const int64_t* ts, const int64_t* val,
                  const int32_t* kh, int64_t n, PRec* part, int64_t mb, uint32_t* rt, uint32_t* rt_t, uint32_t* voffs,
                  uint32_t* srow, uint32_t* scan_tmp, int64_t* sk, int64_t* stt, int64_t* sv, int32_t* skh, DevSide side,
                  Status* st, hipStream_t_ s);
void launch_taint(const DevCfg& c, int64_t wm, const int64_t* key, const int64_t* ts, int64_t n, Status* st,
                  hipStream_t_ s);
// srow: the ordered-path counts per tile, scanned (T), then raw (T): rows P and P + 1 of a partition-major
// batch's scanned histogram
void launch_slow(const DevCfg& c, int64_t wm, const uint32_t* srow, int32_t T, const int64_t* sk,
                 const int64_t* stt, const int64_t* sv, const int32_t* skh, DevTable tb, DevRows out, DevSide side,
                 Status* st, int resume, hipStream_t_ s);
void launch_fire(const DevCfg& c, int64_t wm, DevTable tb, DevRows out, Status* st, hipStream_t_ s);
int64_t pane_nt_floor(const DevCfg& c, int64_t wm);  // host: DevCfg::nt_floor of a launch at watermark wm
// FW_AGG_HLL: fold the batch's records into the registers of their (key, window) entries (after aggregate)
void launch_hll_update(const DevCfg& c, const PRec* part, const uint32_t* offs, int32_t T, int64_t n, DevTable tb,
                       Status* st, hipStream_t_ s);
// FW_AGG_ROW: add the batch's records' columns into the blocks of their (key, window) entries (after aggregate)
void launch_row_update(const DevCfg& c, const PRec* part, const uint32_t* offs, int32_t T, int64_t n, DevTable tb,
                       Status* st, hipStream_t_ s);
// FW_AGG_TDIGEST: compress the batch's values into the digests of their (key, window) entries (after aggregate)
void launch_td_relink(const DevCfg& c, DevTable tb, hipStream_t s);
void launch_tdigest(const DevCfg& c, const PRec* part, const uint32_t* offs, int32_t T, int64_t n, DevTable tb,
                    TdBuf& td, Status* st, hipStream_t_ s);
// FW_COUNT: one batch of count windows (key slots, stable sort by key, fire, ring update); val = the push's values
void launch_count(const DevCfg& c, DevCount& cw, const int64_t* key, const int64_t* val, int64_t n, DevRows out,
                  Status* st, hipStream_t_ s);
size_t count_sort_bytes(int64_t n);
void launch_rehash(const DevCfg& old_c, DevTable old_t, const DevCfg& new_c, DevTable new_t, hipStream_t_ s);
void launch_table_stats(const DevCfg& c, DevTable tb, unsigned long long* out3, hipStream_t_ s);
void launch_reset_regions(const DevCfg& c, DevTable tb, hipStream_t_ s);
// HyperLogLog partials (combining): pass 1 counts each partial's non-zero registers into cnt[0, n) and scans it in
// place (cnt[n] = total; scan_tmp: launch_scan's for n + 1 words); pass 2 writes them at those offsets and frees the
// blocks; the receiver's offsets are the scan of the partials' sum column, then the registers are raised
void launch_hll_extract_counts(const DevCfg& c, PartialCols out, int64_t n, uint32_t* cnt, uint32_t* scan_tmp,
                               hipStream_t_ s);
void launch_hll_extract_regs(const DevCfg& c, PartialCols out, int64_t n, const uint32_t* off, uint32_t* regs,
                             hipStream_t_ s);
void launch_hll_reg_offsets(PartialCols in, int64_t n, uint32_t* off, uint32_t* scan_tmp, hipStream_t_ s);
void launch_hll_push_regs(const DevCfg& c, int64_t wm, PartialCols in, int64_t n, const uint32_t* regs,
                          const uint32_t* off, DevTable tb, Status* st, hipStream_t_ s);
// combining: offs[P+1] = exclusive scan of the regions' live counts (scratch: launch_scan's)
void launch_live_offsets(const DevCfg& c, DevTable tb, uint32_t* offs, uint32_t* scratch, hipStream_t_ s);
void launch_extract(const DevCfg& c, DevTable tb, const uint32_t* offs, PartialCols out, hipStream_t_ s);
void launch_pscatter(const DevCfg& c, int64_t wm, PartialCols in, int64_t n, int32_t T, uint32_t* offs, PartialRec* part,
                     Status* st, hipStream_t_ s);
void launch_pmerge(const DevCfg& c, const PartialRec* part, const uint32_t* offs, int32_t T, DevTable tb, AggProg prog,
                   int resume, Status* st, hipStream_t_ s);
// dense regions: restored rows of key group kg as partials in partition-major runs (prep: partition and internal
// representation of every row, key-group errors counted; then hist, scan and scatter into `part` at offsets
// `hist` ((P + 1) x T, scanned in place)), merged by launch_pmerge
void launch_dt_restore_runs(const DevCfg& c, int32_t kg, StateCols in, int64_t n, int32_t* rp, uint32_t* hist,
                            uint32_t* scan_tmp, PartialRec* tmp, PartialRec* part, Status* st, hipStream_t_ s);
void launch_block_export(const DevCfg& c, const int64_t* blk, int64_t n, uint8_t* acc, hipStream_t_ s);
void launch_pool_take(const DevCfg& c, int32_t h, int32_t take, int64_t bump, int64_t n, int64_t* ids, hipStream_t_ s);
void launch_pool_give(const DevCfg& c, const int64_t* ids, int64_t n, int32_t h, hipStream_t_ s);
void launch_snapshot(const DevCfg& c, DevTable tb, int32_t p0, int32_t np, StateCols out, unsigned long long* count,
                     hipStream_t_ s);
// demand != NULL: count rows per partition (and key-group errors); NULL: insert the rows
// (insertion: round_of[i] = the row's round, rows with the same (key, window) in different rounds; NULL = one)
void launch_restore(const DevCfg& c, int32_t kg, StateCols in, int64_t n, int32_t* demand, DevTable tb, Status* st,
                    const int32_t* round_of, int32_t rounds, hipStream_t_ s);
void launch_key_groups(const int64_t* key, const int32_t* kh, int32_t key_kind, int64_t n, int32_t max_par,
                       int32_t* kg, hipStream_t_ s);
void launch_route(const int64_t* key, const int64_t* ts, const int64_t* val, const int32_t* kh, int32_t key_kind,
                  int64_t n, int32_t max_par, int32_t par, int64_t* ko, int64_t* to, int64_t* vo, int32_t* ho,
                  int64_t* counts, uint32_t* scratch, hipStream_t_ s);
void launch_generate(uint64_t seed, int64_t first, int64_t n, int64_t num_keys, const double* cdf, int64_t ts_base,
                     int64_t rate, int64_t jitter, int64_t* key, int64_t* ts, int64_t* val, int64_t* max_ts,
                     hipStream_t_ s);
}  // namespace fwdev
