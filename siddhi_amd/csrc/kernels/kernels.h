// Host-side launchers of the gfx950 kernels (kernels.hip). All launches are asynchronous on `stream`.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../engine/nfa.h"
#include "../engine/plan.h"

namespace sdg {

// ---- key grouping: stable LSD radix sort of a batch by dense key id ------------------------------------
// Each pass sorts by one digit of <= 8 bits (<= 256 buckets): per-tile digit histogram -> prefix over tiles ->
// stable tile scatter. Inside a tile (4096 events, 256 threads) ranks are stable (wave ballot match over the
// digit bits + per-wave prefix in LDS), the tile is staged in LDS in digit order and every column is written
// out with consecutive lanes on consecutive addresses of one digit run (coalesced), one column at a time.
constexpr int RX_TILE = 8192;     // default (round 6): 32 rows per bucket run on average at 256 buckets, two blocks per CU
constexpr int RX_THREADS = 512;
constexpr int RX_TILE_BIG = 16384;  // 64 rows per run; one 1024-thread block per CU (SDG_RX_TILE=16384, A/B). r3z had it
constexpr int RX_THREADS_BIG = 1024;  // ahead; with compile-time 8-bit digits the small tile wins: C5 key sort 14.63 ->
#ifndef SDG_RX_TILE_DEFAULT           // 13.85 ms per 2^28-row flush (r6u)
#define SDG_RX_TILE_DEFAULT 8192
#endif
constexpr int RX_TILE_DEFAULT = SDG_RX_TILE_DEFAULT;
constexpr int RX_MAXBITS = 8;
constexpr int KG_GROUP = 64;          // tiles per prefix group

struct KeyGroupArgs {
    int64_t n;
    int32_t K;                        // keys are dense ids < K
    const uint32_t* keys;             // [n] input keys (time order)
    // workspace (keygroup_workspace)
    uint32_t* counts;                 // [ntiles * 256]
    uint32_t* gsum;                   // [ngroups * 256]
    uint32_t* tot;                    // [257]
    uint32_t* tmp_keys[2];            // [n] ping-pong key buffers
    uint32_t* tmp_orig[2];            // [n] ping-pong original-row buffers
    void* tmp_cols[2][MAX_COLS + 2];  // [n * width] ping-pong payload buffers
    // outputs
    uint32_t* keys_sorted;            // [n]
    uint32_t* orig_sorted;            // [n] original row of each sorted position
    uint32_t* seg_start;              // [K] first sorted position of key k (0 if absent)
    uint32_t* seg_end;                // [K] one past the last (0 if absent)
    int32_t ncols;                    // payload columns moved with the keys
    const void* src[MAX_COLS + 2];
    void* dst[MAX_COLS + 2];
    uint8_t width[MAX_COLS + 2];      // bytes per element (1, 4 or 8)
    int* key_flag;                    // non-null: set to 1 when some key >= K (the first histogram pass checks)
    const uint32_t* orig_in;          // [n] batch position of each input row (nullptr: the row index itself);
                                      // orig_sorted then holds positions
    // payload column ts32_col (int64 ts) is written as u32 offsets from *ts_base (bucketize: the batch's first ts,
    // an offset past 2^32 sets the mono flag; keygroup: the sorted-view matcher's window base, the first pass
    // converts and sets *ts32_flag for an offset outside [0, 2^32), the later passes move u32), and (bucketize only)
    // the keys as u8 local keys key >> bits into lkey_out instead of keys_sorted (ts32_col < 0 / lkey_out nullptr: off)
    int32_t ts32_col = -1;
    const int64_t* ts_base = nullptr;
    int* ts32_flag = nullptr;
    uint8_t* lkey_out = nullptr;
    // prefix rows (keygroup, the sorted-view matcher's folded carries): rows [0, pre_n) of the input are read from
    // pre_keys / pre_src (8-byte slots per row; a narrower column takes the slot's low bytes), rows [pre_n, n) from
    // keys / src; a prefix row's orig is 0x80000000 | its index. n counts both
    int64_t pre_n = 0;
    const uint32_t* pre_keys = nullptr;
    const void* pre_src[MAX_COLS + 2] = {};
    int32_t no_segments = 0;          // keygroup: skip seg_start / seg_end (the sorted-view matcher finds runs by key)
};
// bytes of workspace for n events; fills the workspace pointers of `a` from `base`
size_t keygroup_workspace(int64_t n, int32_t K, int32_t ncols, const uint8_t* widths);
void keygroup_bind(KeyGroupArgs& a, void* base);
// marks (optional, 4 events): recorded before the histograms, after the prefix kernels of pass 1, after
// the last scatter, after the segment kernel
// *out = ts[0] - 2^31: the base of the sorted view's u32 ts offsets (rows within +-2^31 ms of the batch's first)
void ts_window_base(const int64_t* ts, int64_t* out, hipStream_t stream);
void keygroup(const KeyGroupArgs& a, hipStream_t stream, hipEvent_t* marks = nullptr);

// ---- bucket grouping (fused chain path): ONE radix pass on the key's low `bits` bits --------------------
// Rows of a bucket end up contiguous and in arrival order (stable); key k is in bucket k & (2^bits - 1). The
// pass also checks that the batch's timestamps are non-decreasing in arrival order (mono_flag != 0 otherwise,
// the precondition of the fused matcher's per-bucket time order). Outputs bstart[nb + 1] (bucket row ranges)
// and bseg[nb + 1] (exclusive prefix over buckets of ceil(len / seg_rows): the matcher's block plan).
// marks (optional, 4 events) as keygroup().
// tm (optional, tm_cap >= the fused grid + 2 entries): the time-major block plan (ChainArgs::tm)
void bucketize(const KeyGroupArgs& a, int bits, int ts_col, int* mono_flag, uint32_t* bstart, uint32_t* bseg,
               int seg_rows, hipStream_t stream, hipEvent_t* marks = nullptr, uint32_t* tm = nullptr, int64_t tm_cap = 0);
// one time sub-batch of the fused path (round 6): rows [row0, row0 + n) of the batch described by `a` (its src / keys
// at row 0; a.n ignored), of which the first `own` (a multiple of the bucket tile, bucket_tile()) are the sub-batch's
// own rows and the rest its halo; writes the view at a.dst / lkey_out / orig_sorted from 0, orig = batch row, and
// bstart / bseg (segments over own rows only) / bown (ChainArgs::bown). ts_col's arrival order is checked from row0
// against row0 - 1 as well.
void bucketize_sub(const KeyGroupArgs& a, int bits, int ts_col, int* mono_flag, int64_t row0, int64_t n, int64_t own,
                   uint32_t* bstart, uint32_t* bseg, uint32_t* bown, int seg_rows, hipStream_t stream);
int bucket_tile();
// the halo of every sub-batch but the last must reach past the window of its last own row: flags[5] = 1 when row
// (j + 1) * S + H (if < n) is not later than ts[(j + 1) * S - 1] + within_ms for some j (the host then reruns the flush
// without sub-batches)
void sub_halo_check(const int64_t* ts, int64_t n, int64_t S, int64_t H, int64_t within_ms, int* flags, hipStream_t st);

// ---- chain matcher: `every e1=S0[c0] -> e2=S1[c1] within T` (independent partials) ---------------------
// One block per tile of CM_THREADS * CM_EPT sorted events; the block reserves its output range with one atomic.
constexpr int CM_THREADS = 256;
constexpr int CM_EPT = 8;
constexpr int CM_TILE = CM_THREADS * CM_EPT;
constexpr int CM_HALO = 256;                         // rows staged past the tile (scans continue in HBM beyond)
constexpr int CM_ROWS = CM_TILE + CM_HALO;
constexpr int CM_SCOLS = 2;                          // columns of the state-1 filter staged in LDS
// the part of the plan the chain kernels read, copied into their argument block: ChainArgs is read through a
// __restrict__ const kernel pointer, so these loads are scalar (SMEM) and the values provably wave-uniform
struct ChainSpec {
    int32_t n_states, has_within;
    int64_t within_ms;
    FastPred f0, f1;
    Prog prog0, prog1;                // state filters (bytecode, when f0/f1 are FP_NONE)
    int32_t n_out, n_cols;
    Prog out_prog[MAX_OUT];
    Instr out_ins[MAX_OUT];           // the select expression when it is one OP_LOAD (out_direct)
    uint8_t out_direct[MAX_OUT];
    uint8_t col_kind[MAX_COLS];
    // the e2 filter as a typed scan: `e2.scan_col OP k` (scan_e2_left) or `k OP e2.scan_col`, compared as kind
    // scan_t; k = scan_konst (SCAN_CONST) or e1.e1_col converted to scan_t (SCAN_E1); SCAN_TRUE: no filter;
    // SCAN_GENERIC: f1 / the bytecode per row
    int32_t scan_mode;
    int32_t scan_col, e1_col;
    uint8_t scan_col_kind, e1_col_kind, scan_t, scan_op, scan_e2_left;
    int64_t scan_konst;
};
enum ScanMode : int32_t { SCAN_GENERIC = 0, SCAN_TRUE = 1, SCAN_CONST = 2, SCAN_E1 = 3 };

// XCD-aware block order. The hardware deals consecutive workgroup ids round-robin to the device's XCDs (each with
// its own L2); the kernels that share halo rows or output cache lines between neighbouring blocks remap the block id
// so that each XCD gets a contiguous run of virtual ids. g_xcds is the device's XCD count
// (hipDeviceAttributeNumberOfXccs at engine creation: 8 on MI355X in SPX mode, fewer per device under CPX/DPX
// partitioning); 1 disables the remap. Grids of remapped kernels are rounded up to a multiple of it (xcd_round).
extern int g_xcds;
extern int g_cus;  // the device's CU count (persistent grids)
__host__ __device__ __forceinline__ uint32_t xcd_block(uint32_t bid, uint32_t grid, uint32_t xcds) {
    return xcds > 1 ? (bid % xcds) * (grid / xcds) + bid / xcds : bid;
}
inline int64_t xcd_round(int64_t g) { return g_xcds > 1 ? (g + g_xcds - 1) / g_xcds * g_xcds : g; }

struct ChainArgs {
    ChainSpec sp;
    int32_t xcds;                     // XCD count for the block remap (g_xcds at the flush)
    const Plan* plan;                 // device copy
    const Instr* code;
    const int64_t* consts;
    int64_t n;
    const int64_t* ts;                // sorted view
    const uint8_t* qstream;           // [n] query-stream position of each row (nullptr: single stream 0)
    const uint32_t* key;              // [n] sorted keys (nullptr: unpartitioned, one segment)
    const uint32_t* seg_start;        // [K] (nullptr: unpartitioned)
    const uint32_t* seg_end;          // [K]
    int32_t K;
    const uint32_t* orig;             // [n] sorted -> original row (nullptr: identity)
    const void* cols[MAX_COLS];
    const uint8_t* nulls[MAX_COLS];
    int64_t seq_base;                 // global sequence number of batch row 0
    int32_t s0, s1;                   // query-stream position of state 0 / state 1 events
    // matches
    int64_t out_cap;
    unsigned long long* out_count;
    int64_t* out_ts;
    uint32_t* out_key;                // nullptr: not written
    int64_t* out_vals;                // [n_out][out_cap]
    uint32_t* out_nulls;              // [out_cap] bit per output attribute (written when write_nulls)
    int64_t* out_emit_seq;            // sequence number of the event that completed the match
    int64_t* out_first_seq;           // sequence number of e1
    // partials still pending at the end of the batch
    int64_t carry_cap;
    unsigned long long* carry_count;
    uint32_t* carry_key;
    int64_t* carry_ts;
    int64_t* carry_seq;
    int64_t* carry_vals;              // [n_cols][carry_cap]
    uint32_t* carry_nulls;
    // partials carried in from the previous batch
    int64_t cin_n;
    const uint32_t* cin_key;
    const int64_t* cin_ts;
    const int64_t* cin_seq;
    const int64_t* cin_vals;          // [n_cols][cin_cap]
    const uint32_t* cin_nulls;
    int64_t cin_cap;
    int* flags;                       // [0] overflow, [1] non-monotonic timestamps within a key
    // LDS staging (chain_match_k): columns mirrored in LDS and their slot per column (-1: HBM only)
    int32_t n_stage;
    int32_t stage_col[CM_SCOLS];
    int8_t stage_of[MAX_COLS];
    int32_t lds_stack;                // 1: some filter / select runs the bytecode (needs the LDS stack)
    int32_t generic;                  // 1: bytecode or SCAN_GENERIC needed -> chain_match_k<true>
    int32_t scan_lds;                 // 1: the typed scan's column is staged and has no nulls (LDS-only loop)
    // deque path (chain_deque_k): per-row match results mq[n] (e2 row | MQ_NONE | MQ_CARRY), rows whose lane
    // deque overflowed go to ovf_rows for a forward scan (chain_ovf_k); chain_match_k then only emits
    int32_t deque_mode;               // DQ_OFF / DQ_STACK (x OP top.y pops a suffix) / DQ_ALL (a match completes all)
    int32_t f0_on_x;                  // c0 is `scan_col OP const` (evaluated on the loaded value)
    uint32_t* mq;                     // [n]
    unsigned long long* ovf_count;
    uint32_t* ovf_rows;               // [n]
    // one-key batches (unpartitioned): per 64-row chunk, the largest / smallest converted scan value of its rows that
    // can compare true (not null, not NaN) and whether there is one; a lane's continuation skips the chunks that
    // cannot complete its deque's top (chain_dq_summ_k). nullptr: no summaries
    int64_t* dq_hi;
    int64_t* dq_lo;
    uint8_t* dq_any;
    int64_t* dq_hi8;                  // the same per DQ_GROUP = 8 rows
    int64_t* dq_lo8;
    uint8_t* dq_any8;
    int32_t dq_lane;                  // rows each lane owns (0: DQ_CHUNK); a multiple of DQ_GROUP
    const uint32_t* mq_in;            // chain_match_k: results to emit (nullptr: scan itself)
    int32_t write_nulls;              // 0: no output can be null (out_nulls is not written)
    // fused bucket path (chain_fused_k): the view is bucket-ordered (bucketize), not key-sorted. bstart != nullptr
    // switches chain_carry_k / chain_fovf_k to scanning a key's bucket with a key filter.
    const uint32_t* bstart;           // [nb + 1] bucket row ranges
    // the slim bucket view (bucketize with ts32 / lkey): ts = *ts_base + ts32[r], key = lkey[r] << bbits | bucket;
    // ts / key are nullptr then
    const uint32_t* ts32;
    const int64_t* ts_base;
    const uint8_t* lkey;
    const uint32_t* bseg;             // [nb + 1] block plan (exclusive prefix of segments per bucket)
    int32_t nb, bbits, lbits;         // buckets = 2^bbits; local key = key >> bbits < 2^lbits <= 256
    volatile int64_t* dbg;            // SDG_DEBUG: host-mapped progress trace [block * 4 + wave] (nullptr: off)
    int32_t fu_mode;                  // chain_fused_k: DQ_STACK / DQ_ALL -> chunked deque pass, DQ_OFF -> forward scans
    int32_t fu_skip;                  // SDG_FU_SKIP (phase timing only, results invalid): 1 scan, 2 emit, 4 stop
                                      // after the loads, 8 stop after the LDS regrouping
    int32_t fu_own;                   // chain_fused_k: own (candidate) rows per segment (FU_OWN; one-key batches
                                      // FU_ROWS / 2: a larger halo, as their window spans more rows)
    int32_t fu_check_ts;              // chain_fused_k: check that the staged rows' ts never decrease (one-key
                                      // batches, which no bucket pass checked); flags[3] -> the lane kernels
    int32_t fold;                     // chain_sorted_k: the carried partials are rows of the sorted view (orig =
                                      // 0x80000000 | carry index; keygroup's prefix rows), no chain_carry pass
    // fused bucket path: columns the matcher reads only to emit (no filter reads them, no nulls) stay in arrival
    // order -- the bucket pass does not move them; a view row r reads ocols[c][orig[r]] (col_at)
    uint32_t ocol_mask;
    const void* ocols[MAX_COLS];
    // fused bucket path with ocols: time-major block plan (bucketize): tm[0] = S, the most segments of a bucket (0:
    // bucket-major order), tm[1] = the fewest, tm[2 + s] = blocks of segment index < s over all buckets; block v runs
    // segment s of the r-th bucket that has more than s segments (v < tm[1] * nb: bucket v % nb, segment v / nb)
    const uint32_t* tm;
    // fused path over time sub-batches (round 6, bucketize_sub): the view holds one sub-batch's own rows plus a halo of
    // the following rows that reaches past every own row's window. bown[b]: the end of bucket b's own rows (its
    // segments cover only those; the halo rows are staged and scanned, never candidates). sub_dead: a partial whose
    // key's rows end inside this view with it pending is dead (the halo proves the window passed), not carried --
    // every sub-batch but the flush's last
    const uint32_t* bown;
    int32_t sub_dead;
};
enum DequeMode : int32_t { DQ_OFF = 0, DQ_STACK = 1, DQ_ALL = 2 };
constexpr uint32_t MQ_NONE = 0xFFFFFFFFu, MQ_CARRY = 0xFFFFFFFEu, MQ_OVF = 0xFFFFFFFDu;
constexpr int DQ_THREADS = 256;
constexpr int DQ_CHUNK = 64;                         // consecutive sorted rows per lane
constexpr int DQ_GROUP = 8;                          // rows loaded per step
constexpr int DQ_DEPTH = 8;                          // deque entries per lane (LDS ring); more -> ovf_rows
size_t chain_lds_bytes(const ChainArgs& a);
// deque path: rows -> mq (+ overflow rows resolved by forward scans)
void chain_deque(const ChainArgs& a, const ChainArgs* d_a, hipStream_t stream);
// kernel arguments are read from a device copy (d_a) of `a`: the struct is too large to index as a kernarg
void chain_match(const ChainArgs& a, const ChainArgs* d_a, hipStream_t stream);
void chain_carry(const ChainArgs& a, const ChainArgs* d_a, hipStream_t stream);
// sorted-view matcher (radix path): LDS-staged blocks of FU_ROWS sorted rows, chunked deque + forward scans, matches
// emitted in the kernel; chain_sovf then resolves the partials whose key continues past their block's staged rows
void chain_sorted(const ChainArgs& a, const ChainArgs* d_a, hipStream_t stream);
void chain_sovf(const ChainArgs& a, const ChainArgs* d_a, hipStream_t stream);

// ---- fused bucket matcher -------------------------------------------------------------------------------
// One block per segment of FU_OWN rows of one bucket: the segment plus FU_HALO following rows of the bucket
// are staged in LDS and regrouped by local key there (stable counting sort), so each candidate's forward scan
// walks its key's run in LDS. A scan that leaves the staged rows before the bucket ends goes to chain_fovf_k
// (the same scan over the bucket in HBM, key-filtered); one that reaches the bucket end is carried.
// Preconditions (host): partitioned, one stream, two states, `within`, typed e2 scan without nulls, FastPred
// e1 filter, plain-attribute selects, K <= 2^16, batch timestamps non-decreasing (checked by bucketize).
#ifndef SDG_FU_THREADS
#define SDG_FU_THREADS 512  // (A/B builds: 1024 -> 4096 staged rows per block, 2 blocks of ~78 KB LDS per CU)
#endif
constexpr int FU_THREADS = SDG_FU_THREADS;
#ifndef SDG_FU_PT
#define SDG_FU_PT 4  // (A/B builds: 8 -> 4096 staged rows per 512-thread block, 2 blocks per CU)
#endif
constexpr int FU_PT = SDG_FU_PT;                     // staged rows per lane (= the deque chunk)
constexpr int FU_ROWS = FU_THREADS * FU_PT;          // 2048 rows in LDS
#ifndef SDG_FU_DQ
#define SDG_FU_DQ 4
#endif
// deque chunk: positions per lane in the monotone-deque pass (FU_ROWS / FU_DQ lanes work, the other waves idle).
// Longer chunks pay a lane's continuation over the key's following rows (~ the window) once per more rows, but
// lengthen the block's critical path: measured 8 -> 2.85 ms vs 4 -> 2.65 ms (r1ab), so the pass is latency-bound
constexpr int FU_DQ = SDG_FU_DQ;
#ifndef SDG_FU_HALO
#define SDG_FU_HALO 512  // ~1.3 s of a bucket at C2 (> T)
#endif
constexpr int FU_HALO = SDG_FU_HALO;
constexpr int FU_OWN = FU_ROWS - FU_HALO;            // candidate rows per block
// grid size for n rows in nb buckets (a multiple of g_xcds: the XCD remap needs it)
int64_t chain_fused_grid(int64_t n, int nb, int own = FU_OWN);
void chain_fused(const ChainArgs& a, const ChainArgs* d_a, int64_t grid, hipStream_t stream);
// whether chain_fused has the arrival-order-column build for this scan (ChainArgs::ocols; sp and fu_check_ts set)
bool chain_fused_ocols_ok(const ChainArgs& a);
// the rows chain_fused_k handed over (ovf_rows / ovf_count): key-filtered bucket scans in HBM, emitted directly
void chain_fovf(const ChainArgs& a, const ChainArgs* d_a, hipStream_t stream);

// ---- generic keyed NFA (nfa.h): one lane per partition key walks that key's events in order --------------
struct NfaArgs {
    const Plan* plan;
    const Instr* code;
    const int64_t* consts;
    int64_t n;
    const int64_t* ts;                // sorted view
    const uint8_t* qstream;           // nullptr: single stream 0
    const uint32_t* vrank;            // range partitions: the range of each view row; broadcast rows: the key's
                                      // rank in getPartitionKeys() order (nullptr: none)
    const uint32_t* seg_start;        // [K] (nullptr: unpartitioned, K == 1, one segment [0, n))
    const uint32_t* seg_end;
    int32_t K;
    const uint32_t* orig;             // sorted -> batch position (nullptr: pos_off + row)
    int64_t pos_off;
    const void* cols[MAX_COLS];
    const uint8_t* nulls[MAX_COLS];
    int64_t seq_base;                 // sequence number of batch position 0
    uint8_t* arena;                   // [K][L.bytes], zero-initialised on allocation, persists across batches
    uint8_t* arena2;                  // second copy (nullptr: the run updates `arena` in place). With two, a run
                                      // copies the key's committed state to the other copy and works there, so a
                                      // key can be rerun from its batch-start state until nfa_commit flips it
    uint8_t* cur;                     // [K] which copy holds the committed state (arena2 != nullptr)
    uint8_t* ran;                     // [K] set for every key this run touched (arena2 != nullptr)
    nfa::Layout L;
    int64_t out_cap;
    unsigned long long* out_count;
    int64_t* out_ts;
    uint32_t* out_key;
    int64_t* out_vals;                // [n_out][out_cap]
    uint32_t* out_nulls;
    int64_t* out_emit_seq;            // sequence number of the event whose processing emitted the match
    int64_t* out_sub;                 // emission ordinal within that event (timer matches: negative)
    uint8_t* out_round;               // [out_cap] scheduler round that produced the record (nullptr: not written)
    uint8_t round;
    int* flags;                       // [0] output overflow, [2] arena overflow, [5] scheduler log overflow
    // timers (queries with absent states)
    nfa::TimerIn T;
    // @purge: per-key last activity (persistent, INT64_MIN = never), the clock, the purge window. A run reads the
    // batch-start readings (last_seen_in) and writes the run's (last_seen), so any key can rerun from the batch start
    int64_t* last_seen;               // nullptr: the query's partition does not purge
    const int64_t* last_seen_in;
    uint8_t* out_flags;               // [out_cap] per record: aggregator reset before it (nullptr: not recorded)
    uint8_t* agg_reset;               // [K] set for a key purged after its last record of the run (nullptr: none)
    // idle keys (nfa.h to_idle / from_idle; nullptr unless the query reclaims arenas): arenas, cur / ran bits are
    // indexed by slot, slot_of maps keys to slots
    const int32_t* slot_of;           // [K] arena slot of key k; -1 never seen, -2 idle (its record in idle_rec)
    const uint8_t* init_from;         // [slots] 1: the slot's key starts fresh in this batch, 2: from its idle record
    const uint8_t* idle_rec;          // [K][idle_bytes]
    uint8_t* idle_out;                // [slots][idle_bytes] the record of a key that ended the run idle
    uint8_t* releasable;              // [slots] 1: the slot's key ended idle (the slot returns to the pool at commit)
    int32_t idle_bytes;
    const int64_t* purge_clk;
    int64_t purge_from, purge_idle;
    // rerun mode: run only list[0..nlist) with the explicit fire lists fires[fire_off[i] .. fire_off[i + 1])
    const uint32_t* list;
    int32_t nlist;
    const uint32_t* fire_off;
    const nfa::TimerFire* fires;
    // keys whose run overflowed the arena (the host takes them over when the layout is at its largest)
    uint32_t* ovf_keys;               // [ovf_cap] (nullptr: not recorded)
    unsigned int* ovf_count;
    int32_t ovf_cap;
};
// ---- register sequence kernel (seq3.hip): SEQUENCE `every e1=S[f1], e2=S[f2]<m:n>, e3=S[f3]` ------------------
// Per partition key the reference holds at most one partial waiting at e2 (Q) and one at e3 (P; the same object as Q
// while the count state both forwards and keeps it): SEQUENCE addState keeps one state event per newAndEvery list
// (StreamPreStateProcessor.java:214-227, CountPreStateProcessor.java:97-125) and every pending list is cleared before
// each event (resetState :288-305). So a key's whole state is two partials of three events each (e1, e2[0],
// e2[last]) -- registers instead of an arena. tests/seq3_model.py states the model; tests/test_seq3_model.py pins it
// against the oracle.
constexpr int S3_MAX_COLS = 4;   // physical columns stored per event
constexpr int S3_MAX_OUT = 8;
constexpr int S3_STAGE = 256;    // output records staged in LDS per wave (one global reservation per flush of them)
enum S3Src : int8_t { S3_NULL = -1, S3_E1 = 0, S3_E2F = 1, S3_E2L = 2, S3_Y = 3 };
struct S3Operand {
    int8_t src;      // S3Src: which event of the partial (Y = the event being processed)
    uint8_t col;     // physical column
    uint8_t kind;    // its kind
    uint8_t pad;
};
struct S3Pred {      // FastPred with its operands resolved for one processor's context
    uint8_t kind;    // FP_TRUE / FP_CONST / FP_SLOT
    uint8_t op, t, pad;
    S3Operand a, b;
    int64_t konst;
};
struct Seq3Spec {
    int32_t nc;                      // physical columns (<= S3_MAX_COLS), stored for every event of a partial
    int32_t n_out;
    int32_t min_count, max_count;    // max INT32_MAX: unbounded
    int32_t has_within;              // `within T`: a partial whose e1 is more than T away is dropped before the event
    int64_t within_ms;
    uint8_t col_kind[S3_MAX_COLS];
    S3Pred f[3];                     // e1 filter (Y = the e1 candidate), e2 filter (E1, E2F, Y = e2[last]),
                                     // e3 filter (E1, E2F, E2L of P, Y = e3)
    S3Operand out[S3_MAX_OUT];       // select items, resolved like the e3 filter
};
struct Seq3Args {
    Seq3Spec sp;
    int64_t n;
    const int64_t* ts;                // sorted view (nullptr: not sorted; the output ts is ts_view[orig[r]])
    const int64_t* ts_view;           // arrival-order ts of the query's view rows
    const uint32_t* seg_start;        // [K] (nullptr: unpartitioned, one key over [0, n))
    const uint32_t* seg_end;
    int32_t K;
    const uint32_t* orig;             // sorted -> batch position (nullptr: pos_off + row)
    int64_t pos_off;
    int64_t seq_base;
    const void* cols[S3_MAX_COLS];
    const uint8_t* nulls[S3_MAX_COLS];
    // per-key state, SoA with stride kcap (persistent; zeros = no partial): hdr bit 0 P, bit 1 Q, bit 2 P is Q,
    // bits 8..31 Q's e2 count (saturating); pn / qn null bits of P / Q (e1 bits 0.., e2[0] 8.., e2[last] 16..);
    // vals[(g * nc + c) * kcap + k], g = P.e1, P.e2[0], P.e2[last], Q.e1, Q.e2[0], Q.e2[last]
    uint32_t* st_hdr;
    uint32_t* st_pn;
    uint32_t* st_qn;
    int64_t* st_vals;
    int64_t* st_ts;                   // [2][kcap] e1 timestamps of P and Q (has_within)
    int64_t kcap;
    // outputs (at most one record per event: out_cap >= n never overflows)
    int64_t out_cap;
    unsigned long long* out_count;
    int64_t* out_ts;
    uint32_t* out_key;
    int64_t* out_vals;                // [n_out][out_cap]
    uint32_t* out_nulls;
    int64_t* out_emit_seq;
    int64_t* out_sub;
    int* flags;                       // [0] output overflow
};
void seq3_run(const Seq3Args& a, const Seq3Args* d_a, hipStream_t stream);

// a: host copy (launch geometry); d_a: device copy the kernel reads. Layouts of at most NFA_LDS_BUDGET /
// NFA_LDS_MIN_LANES bytes per key run with the arenas staged in LDS (nfa_lds_k: one wave per block, lanes =
// NFA_LDS_BUDGET / bytes keys per wave, four blocks per CU); larger ones in HBM (nfa_k)
constexpr int64_t NFA_LDS_BUDGET = 36 * 1024;
constexpr int NFA_LDS_MIN_LANES = 8;
int nfa_lds_lanes(const nfa::Layout& L);
void nfa_run(const NfaArgs& a, const NfaArgs* d_a, hipStream_t stream);
// arena growth: the committed copy of every key (arena2 && cur[k] ? arena2 : arena) into `dst` in layout Ld
void nfa_migrate(const Plan* plan, const uint8_t* arena, const uint8_t* arena2, const uint8_t* cur,
                 const nfa::Layout& Ls, uint8_t* dst, const nfa::Layout& Ld, int64_t K, hipStream_t stream);
// double-buffered arenas: flip `cur` of every key a run touched (`ran`), clearing `ran`
void nfa_commit(uint8_t* cur, uint8_t* ran, int64_t K, hipStream_t stream);
// idle keys: the pool of arena slots
struct SlotPool {
    int32_t* slot_of;                 // [K]
    uint8_t* idle_rec;                // [K][idle_bytes]
    int32_t* slot_key;                // [slots] key of each assigned slot
    uint8_t* init_from;               // [slots]
    uint8_t* releasable;              // [slots]
    uint8_t* idle_out;                // [slots][idle_bytes]
    int32_t* free_slots;              // [slots] stack of free slot ids
    unsigned int* counters;           // [0] free stack top, [1] keys needing a slot (nfa_slots_need)
    int32_t idle_bytes;
};
// keys with rows in this batch but no slot (seg: the key segments; nullptr + K 1: one key) -> counters[1]
void nfa_slots_need(const SlotPool& sp, const uint32_t* seg_start, const uint32_t* seg_end, int64_t K, hipStream_t st);
// give each such key a slot from the free stack (the host made sure there are enough)
void nfa_slots_assign(const SlotPool& sp, const uint32_t* seg_start, const uint32_t* seg_end, int64_t K, hipStream_t st);
// nfa_commit for slot-indexed arenas, then every slot whose key ended idle: record saved, slot back to the pool
void nfa_commit_slots(const SlotPool& sp, uint8_t* cur, uint8_t* ran, int64_t slots, hipStream_t st);

// delivery order of n match records (order.hip): perm = the record indices sorted by (emit - emit_base as u32,
// sub - sub_bias as a sub_bits-bit key: 48, or 64 when a delivery rank sits in bits 40..62 -- range partitions and
// broadcast rows); both sorts cover only the key range the records use (measured first: one small read-back);
// work = order_workspace(n) bytes
size_t order_workspace(int64_t n);
// emit_span: the flush's positions (emit - emit_base < emit_span; 0: unknown, measured)
void order_records(const int64_t* emit, const int64_t* sub, int64_t n, int64_t emit_base, int64_t emit_span,
                   int64_t sub_bias, int sub_bits,
                   void* work, size_t work_bytes, uint32_t** perm_out, hipStream_t stream);
void gather_i64(const int64_t* src, const uint32_t* perm, int64_t n, int64_t* dst, hipStream_t stream);
// the ordered export in one pass after the sort by emitting event (order.hip): each record's run rank and its columns
// straight to its slot, the emitting position written from the sorted key (seq_dst, may be nullptr); work =
// order_workspace(n). false: a run longer than the rank pass handles -- use order_records + gather_cols_i64
bool order_export(const int64_t* emit, const int64_t* sub, int64_t n, int64_t emit_base, int64_t emit_span,
                  const int64_t* const* src, int64_t* const* dst, int ncol, int64_t* seq_dst, void* work,
                  hipStream_t stream);
// dst[c][i] = src[c][perm[i]] for ncol int64 columns, through a packed row-major copy (work = gather_cols_workspace)
constexpr int GATHER_MAX_COLS = 16;
size_t gather_cols_workspace(int64_t n, int ncol);
void gather_cols_i64(const int64_t* const* src, int64_t* const* dst, int ncol, const uint32_t* perm, int64_t n,
                     void* work, hipStream_t stream);
void gather_u32(const uint32_t* src, const uint32_t* perm, int64_t n, uint32_t* dst, hipStream_t stream);
void gather_u8(const uint8_t* src, const uint32_t* perm, int64_t n, uint8_t* dst, hipStream_t stream);

// the selector's post pass (order.hip): aggregators per key in delivery order, select items over them, having
struct SelPostArgs {
    const Plan* plan;                 // device copy
    const Instr* code;
    const int64_t* consts;
    int64_t n;                        // records, in delivery order
    int64_t* vals;                    // [n_out][vstride]: emission columns in, aggregate / post columns out
    int64_t vstride;
    uint32_t* nulls;                  // [n] null bits (updated)
    uint8_t* pass;                    // [n] having result
    int64_t* agg_state;               // [K][n_agg][2], persistent per partition key
    const uint32_t* perm;             // set by select_post
    const uint32_t* key_sorted;
    const uint8_t* reset;             // [n] 1: the record's key was purged since its previous record (nullptr: none)
};
size_t select_post_workspace(int64_t n);
// key: [n] partition key ids < 2^kbits (nullptr / kbits 0: unpartitioned, one run)
void select_post(SelPostArgs a, const uint32_t* key, int kbits, void* work, hipStream_t stream);
// keys flagged in flags[K] (purged after their last record): aggregator states zeroed, flags cleared
void agg_reset(int64_t* agg_state, int n_agg, uint8_t* flags, int64_t K, hipStream_t stream);

// ---- device-side batch view of mixed pushes (ingest.hip) ------------------------------------------------------
constexpr int MV_MAX_STREAMS = 64;
constexpr int MV_MAX_ATTRS = 64;
struct MixedViewArgs {
    int64_t n;                                // rows of the mixed chunk
    int64_t pos0;                             // batch position of its row 0
    const int32_t* streams;                   // [n] app stream of each row
    const int64_t* ts;                        // [n]
    const int64_t* slots[MV_MAX_ATTRS];       // [attr][n] 64-bit slots (sdg_push_mixed)
    const uint8_t* slot_nulls[MV_MAX_ATTRS];  // [attr][n] or nullptr
    int8_t qpos[MV_MAX_STREAMS];              // app stream -> the query's stream position (-1: not read)
    int32_t partitioned;
    int32_t key_attr[MAX_STATES];             // [query stream] partition key attribute
    uint8_t key_kind[MAX_STATES];
    int32_t n_cols;
    int8_t col_attr[MAX_STATES][MAX_COLS];    // [query stream][physical column] attribute or -1
    uint8_t col_width[MAX_COLS];
    // outputs: the query's view rows of this chunk (arrival order)
    int64_t* out_ts;
    uint32_t* out_pos;                        // batch position
    uint8_t* out_qs;                          // query stream position (nullptr: single stream)
    int64_t* out_key;                         // key value (key table encoding; string ids) if partitioned
    void* out_cols[MAX_COLS];
    uint8_t* out_nulls[MAX_COLS];             // nullptr: no null possible in the column
};
size_t mixed_view_workspace(int64_t n);
// the chunk's view row count into *d_total (device); then the rows (work must be kept between the two calls)
void mixed_view_count(const MixedViewArgs& a, const MixedViewArgs* d_a, void* work, int64_t* d_total, hipStream_t st);
void mixed_view_write(const MixedViewArgs& a, const MixedViewArgs* d_a, void* work, hipStream_t st);
void narrow_u32(const int64_t* src, int64_t n, uint32_t* dst, hipStream_t st);

// broadcast rows of a stream without a partition key (ingest.hip; PartitionStreamReceiver.send(ComplexEvent) :274-283):
// the host view holds ONE placeholder row per such event; this expands it into one row per key of the key order the
// event saw (getPartitionKeys(), engine/keyorder.h), ranked by its place there, and moves every other row to its
// place in the expanded view: row r of the compact view lands at off[r] (exclusive prefix of the rows' widths)
constexpr int BX_MAX_COLS = MAX_COLS;
constexpr uint32_t BX_PLACEHOLDER = 0xFFFFFFFFu;  // the compact key of a placeholder row
struct BcastExpandArgs {
    int64_t n;                       // compact rows
    const uint32_t* off;             // [n + 1] output row of each compact row (off[n] = expanded rows)
    int64_t nph;                     // placeholder rows
    const uint32_t* ph_row;          // [nph] their compact rows
    const uint32_t* ph_ord;          // [nph] start of the key order they saw in `ord`
    const uint32_t* ph_k;            // [nph] its length
    const uint32_t* ord;             // concatenated key orders (dense key ids)
    const int64_t* ts;
    const uint32_t* vpos;
    const uint8_t* qs;               // nullptr: one stream
    const uint32_t* key;
    const uint32_t* vrank;           // (ranked view: vrank of the keyed rows; placeholders get their rank)
    int ncols;
    uint8_t width[BX_MAX_COLS];
    const void* cols[BX_MAX_COLS];
    const uint8_t* nulls[BX_MAX_COLS];  // nullptr: no nulls in the column
    int64_t* o_ts;
    uint32_t* o_vpos;
    uint8_t* o_qs;
    uint32_t* o_key;
    uint32_t* o_vrank;
    void* o_cols[BX_MAX_COLS];
    uint8_t* o_nulls[BX_MAX_COLS];
};
void bcast_expand(const BcastExpandArgs& a, int64_t kmax, hipStream_t st);

// device partition key table for integral partition attributes (keytab.hip): value -> dense key id
// one slot = 16 B (key, id, first row) so that a probe's key compare and its id read touch one cache line (round 5:
// the separate key / id arrays cost two dependent random reads per row)
struct KtSlot {
    int64_t key;      // KT_EMPTY: free (slot cap holds the value KT_EMPTY itself: key = 1 when used)
    uint32_t id;      // id + 1 (0: new in this batch)
    uint32_t first;   // a new key's first row
};
struct KeyTab {
    KtSlot* slots;    // [cap + 1]
    uint64_t mask;    // cap - 1 (cap a power of two)
    uint64_t cap;
};
void kt_clear(const KeyTab& t, hipStream_t st);
void kt_load(const KeyTab& t, const int64_t* vals, uint32_t id0, int64_t n, int* flags, hipStream_t st);
void kt_probe(const KeyTab& t, const void* col, int kind, int64_t n, uint32_t* out, unsigned long long* new_count,
              unsigned long long limit, int* flags, hipStream_t st);
void kt_collect(const KeyTab& t, unsigned long long* pairs, int64_t* vals, unsigned long long* cnt, int64_t cap_out,
                hipStream_t st);
void kt_assign(const KeyTab& t, const uint32_t* slots, uint32_t id0, int64_t m, hipStream_t st);
void kt_fix(const KeyTab& t, const void* col, int kind, int64_t n, uint32_t* out, hipStream_t st);

// G-way merge of sorted runs (merge.hip, the ordered result gather on rank 0): keys[r] (int64, non-decreasing) of
// lens[r] records; cols[r * ncols + c] their payload columns of widths[c] bytes; the merged keys / columns in
// (key, run, index) order. Synchronous on `stream` (it reads the runs' end keys back to size the sample sort).
constexpr int MG_MAX_RUNS = 32;
constexpr int MG_MAX_COLS = 16;
void merge_runs_device(int G, const int64_t* const* keys, const int64_t* lens, int ncols, const void* const* cols,
                       const uint8_t* widths, int64_t* out_keys, void* const* out_cols, hipStream_t stream);

}  // namespace sdg
