// Host-side launchers of the gfx950 kernels (kernels.hip). All launches are asynchronous on `stream`.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../engine/plan.h"

namespace sdg {

// ---- key grouping: stable counting sort of a batch by dense key id -------------------------------------
// hist (one wave per chunk, LDS counters) -> per-key prefix over chunks -> stable scatter (one wave per chunk;
// lanes with equal keys are ranked by a ballot match over the key bits, so order inside a key is the
// arrival order). Columns are moved by the scatter (coalesced reads, per-key runs of writes).
constexpr int KG_CHUNK = 65536;       // events per histogram/scatter wave
constexpr int KG_MAXK = 16384;        // key space handled by the LDS-counter path
constexpr int KG_GROUP = 64;          // chunks per prefix group

struct KeyGroupArgs {
    int64_t n;
    int32_t K;
    int32_t nchunks;
    const uint32_t* keys;             // [n] dense key ids (< K)
    uint32_t* counts;                 // [nchunks * K] workspace (becomes per-chunk start offsets)
    uint32_t* gsum;                   // [ngroups * K] workspace
    uint32_t* seg_start;              // [K + 1] out: first sorted position of key k; seg_start[K] = n
    uint32_t* keys_sorted;            // [n] out
    uint32_t* orig_sorted;            // [n] out: original row of each sorted position
    int32_t ncols;                    // columns moved with the keys
    const void* src[MAX_COLS + 2];
    void* dst[MAX_COLS + 2];
    uint8_t width[MAX_COLS + 2];      // bytes per element (1, 4 or 8)
};
size_t keygroup_workspace(int64_t n, int32_t K, int32_t* nchunks, size_t* counts_bytes, size_t* gsum_bytes);
// marks (optional, 4 events): recorded before hist, after hist, after the prefix kernels, after the scatter
void keygroup(const KeyGroupArgs& a, hipStream_t stream, hipEvent_t* marks = nullptr);

// ---- chain matcher: `every e1=S0[c0] -> e2=S1[c1] within T` (independent partials) ---------------------
struct ChainArgs {
    const Plan* plan;                 // device copy
    const Instr* code;
    const int64_t* consts;
    int64_t n;
    const int64_t* ts;                // sorted view
    const uint8_t* qstream;           // [n] query-stream position of each row (nullptr: single stream 0)
    const uint32_t* key;              // [n] sorted keys (nullptr: unpartitioned, one segment)
    const uint32_t* seg_start;        // [K + 1] (nullptr: unpartitioned)
    const uint32_t* orig;             // [n] sorted -> original row (nullptr: identity)
    const void* cols[MAX_COLS];
    const uint8_t* nulls[MAX_COLS];
    int64_t seq_base;                 // global sequence number of batch row 0
    int32_t s0, s1;                   // query-stream position of state 0 / state 1 events
    // matches
    int64_t out_cap;
    unsigned long long* out_count;
    int64_t* out_ts;
    uint32_t* out_key;
    int64_t* out_vals;                // [n_out][out_cap]
    uint32_t* out_nulls;              // [out_cap] bit per output attribute
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
};
void chain_match(const ChainArgs& a, hipStream_t stream);
void chain_carry(const ChainArgs& a, hipStream_t stream);

}  // namespace sdg
