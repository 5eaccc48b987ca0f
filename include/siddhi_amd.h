/* siddhi_amd — MI355X engine for Siddhi's pattern/sequence NFA path: the drop-in C-ABI.
 *
 * The pattern path behind this header runs on the GPU (gfx950 HIP kernels); there is no CPU fallback for a query or a
 * flush (no device => sdg_compile fails with SDG_ERR_DEVICE). Two bounded cases run parts of a flush on the host with
 * the engine's own NFA code (never the test oracle), and sdg_stats.host_rows counts the rows they processed:
 *   - a partition key that outgrows the device arena's 4096 partial matches spills to a host arena and its rows run
 *     there from then on (sdg_stats.spilled_keys);
 *   - absent-state (timer) queries: a key whose results the scheduler's cross-key timer collapse reorders beyond what
 *     a device rerun reproduces is replayed on the host (sdg_stats.sched_host_keys).
 * The ABI is what a JNI / Panama FFM binding of the reference's API would call (INTEGRATION.md shows the bindings):
 *
 *   sdg_compile          <- SiddhiManager.createSiddhiAppRuntime(String)
 *                           (modules/siddhi-core/src/main/java/io/siddhi/core/SiddhiManager.java:93-96)
 *   sdg_stream_index /   <- SiddhiAppRuntime.getInputHandler(String) + the stream definition
 *   sdg_stream_schema       (core/SiddhiAppRuntimeImpl.java:414)
 *   sdg_push             <- InputHandler.send(long, Object[]) for one stream, columnar, one call per row
 *                           (core/stream/input/InputHandler.java:59-70); events keep their call order
 *   sdg_push_events      <- InputHandler.send(Event[]) (:85-95: the clock moves to the last event first)
 *   sdg_push_device      <- the same for event columns already resident in HBM (device pointers)
 *   sdg_advance_time     <- TimestampGeneratorImpl.setCurrentTimestamp (playback clock, util/timestamp/
 *                           TimestampGeneratorImpl.java:105-122) / the wall clock of a live app
 *   sdg_start            <- SiddhiAppRuntime.start() (core/SiddhiAppRuntimeImpl.java:440)
 *   sdg_flush            <- the receivers' per-event processing of everything pushed so far
 *                           (core/query/input/ProcessStreamReceiver.java:98-179 -> state processors)
 *   sdg_poll             <- QueryCallback.receive(long, Event[], Event[]) / StreamCallback.receive(Event[])
 *                           (core/query/output/callback/QueryCallback.java:60-105,
 *                            core/stream/output/StreamCallback.java:93-129), columnar
 *   sdg_snapshot /       <- SiddhiAppRuntime.snapshot() / restore(byte[]), persist() / restoreRevision()
 *   sdg_restore             (core/SiddhiAppRuntimeImpl.java:677-737)
 *   sdg_snapshot_states  <- the StreamPreState maps SnapshotService collects (StreamPreStateProcessor.java:450-469)
 *   sdg_destroy          <- SiddhiAppRuntime.shutdown()
 *
 * Conventions (mirroring the reference): compile errors are returned as status codes with a thread-local
 * message (SiddhiAppCreationException / SiddhiAppValidationException / OperationNotSupportedException); one
 * handle is single-threaded (the reference serialises a query under patternSyncObject); the engine owns the
 * copies it makes of pushed data; poll results are valid until the next sdg_poll / sdg_destroy. Results are never
 * dropped: a flush (explicit, or the automatic one sdg_push runs when batch_capacity events are buffered) appends
 * to the query's backlog, and sdg_poll hands out the whole backlog. A flush consumes its batch even when it fails
 * (the error names the query); queries flushed before the failing one keep their results.
 *
 * Value encoding of columns: INT int32, LONG int64, FLOAT float, DOUBLE double, BOOL uint8, STRING uint32
 * (ids from sdg_intern: equal strings <=> equal ids). Nulls: optional per-column uint8 arrays (1 = null).
 */
#ifndef SIDDHI_AMD_H
#define SIDDHI_AMD_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

enum sdg_status {
    SDG_OK = 0,
    SDG_ERR_PARSE = 1,        /* SiddhiParserException */
    SDG_ERR_VALIDATION = 2,   /* SiddhiAppValidationException / SiddhiAppCreationException */
    SDG_ERR_UNSUPPORTED = 3,  /* OperationNotSupportedException (outside the accelerated subset) */
    SDG_ERR_ARG = 4,
    SDG_ERR_DEVICE = 5,       /* HIP error or no gfx950 device */
    SDG_ERR_CAPACITY = 6      /* a bounded device structure overflowed (reported, never silently dropped) */
};

enum sdg_type { SDG_INT = 0, SDG_LONG = 1, SDG_FLOAT = 2, SDG_DOUBLE = 3, SDG_BOOL = 4, SDG_STRING = 5 };

typedef struct sdg_engine sdg_engine;

typedef struct sdg_opts {
    int32_t device;            /* HIP device ordinal (one engine per GPU) */
    int64_t batch_capacity;    /* max events buffered between flushes (0 = default 1<<24) */
    int32_t max_partials;      /* per-key partial-match slots the generic NFA starts with (0 = default 8; the arenas
                                  double on overflow up to 4096; a key past that continues on the host in an arena
                                  of 32-bit indices -- sdg_stats.spilled_keys --, except in queries with absent
                                  states, whose flush then fails with SDG_ERR_CAPACITY) */
    int32_t flags;             /* SDG_COMPILE_ONLY: parse + lower only, no device (introspection on hosts
                                  without a GPU; push/flush then fail with SDG_ERR_DEVICE) */
} sdg_opts;
#define SDG_COMPILE_ONLY 1
#define SDG_FORCE_GENERIC 2    /* run every query on the generic keyed-NFA kernel (testing: both kernels on one query) */
#define SDG_NO_FUSED 4         /* chain path: always key-sort with the full radix (testing: both chain kernels on one query) */
#define SDG_NO_SEQ3 8          /* sequences of the seq3 shape on the generic keyed NFA instead (testing: both kernels) */
#define SDG_NO_SORTED 64       /* chain path past the fused bucket matcher: the lane deque kernels instead of the
                                  LDS-staged sorted-view matcher (testing: both kernels on one query) */
#define SDG_SCHED_EXACT 16     /* absent states: always run the scheduler's exact pass, even when the device reruns
                                  reproduce the optimistic pass (testing: pins the exact pass against the oracle) */
#define SDG_SCHED_HOST 32      /* absent states: no optimistic pass / device rerun; the exact pass runs over the
                                  ideal-order device run and replays every key it orders differently on the host
                                  (testing: pins the host replay KeyRun against the oracle) */

typedef struct sdg_out {
    int64_t n;                 /* output events */
    const int64_t* ts;         /* [n] event timestamps (StateEvent timestamp) */
    const uint8_t* expired;    /* [n] 1 = removeEvents / expired */
    int32_t n_attrs;           /* output attributes (select list order) */
    const int32_t* types;      /* [n_attrs] sdg_type */
    const int64_t* const* values; /* [n_attrs][n] 64-bit payload (float/double as bit patterns) */
    const uint8_t* const* nulls;  /* [n_attrs][n] 1 = null */
    const int64_t* event_seq;  /* [n] position (from 0, over every pushed event of every stream and every
                                  sdg_advance_time point) of the input event whose processing emitted the row; an
                                  absent state's timer match carries the position whose clock advance fired it */
} sdg_out;

int sdg_compile(const char* siddhi_app, const sdg_opts* opts, sdg_engine** out);
void sdg_destroy(sdg_engine* e);
const char* sdg_last_error(void);

int sdg_stream_index(sdg_engine* e, const char* stream_id);
int sdg_stream_schema(sdg_engine* e, int stream, int32_t* n_attrs, const int32_t** types);
int sdg_num_queries(sdg_engine* e);
/* device path chosen for a query: 0 = chain kernel (independent partials), 1 = generic keyed NFA, 2 = register
 * sequence kernel (SEQUENCE `every e1=S[..], e2=S[..]<m:n>, e3=S[..]`, seq3.hip) */
int sdg_query_path(sdg_engine* e, int query);
/* what a multi-GPU deployment needs to know about a query (siddhi_amd/shard.py ShardedAppRuntime): */
#define SDG_Q_PARTITIONED 1    /* partition with (...): keys are independent, the query shards by key hash */
#define SDG_Q_TIMERS 2         /* absent states: the reference's Scheduler collapses due timers across ALL keys
                                  (Scheduler.java:75-98), so key shards on different GPUs would change the result */
#define SDG_Q_BROADCAST 4      /* a stream of the query has no partition key: its events go to every key of the partition
                                  in one global key order (PartitionStreamReceiver.java:274-283), across shards */
int sdg_query_flags(sdg_engine* e, int query);
/* how a partitioned query keys a stream (PartitionStreamReceiver / ValuePartitionExecutor): the attribute index of a
 * value partition, -2 range partitions, -3 no key (broadcast), -1 the query does not read the stream or is not
 * partitioned. A multi-GPU router shards the stream's events by the hash of that attribute's toString. */
int sdg_query_key_attr(sdg_engine* e, int query, int stream);
/* 1 when the query reads the stream (one of its pattern states is on it), else 0: a multi-GPU router sends a stream
 * that an unpartitioned query reads whole to one GPU */
int sdg_query_reads(sdg_engine* e, int query, int stream);
const char* sdg_query_name(sdg_engine* e, int query);
const char* sdg_query_target(sdg_engine* e, int query);
int sdg_query_output_schema(sdg_engine* e, int query, int32_t* n_attrs, const int32_t** types,
                            const char* const** names);
uint32_t sdg_intern(sdg_engine* e, const char* s, size_t len);
const char* sdg_string(sdg_engine* e, uint32_t id);
/* sdg_intern for n strings at once (a binding's per-batch dictionary fill; C5's 10^7 partition keys per GPU):
 * string i is bytes[offsets[i] .. offsets[i + 1]), offsets has n + 1 entries; its id goes to ids[i] */
int sdg_intern_many(sdg_engine* e, int64_t n, const char* bytes, const int64_t* offsets, uint32_t* ids);

/* columnar host batch for ONE stream: ts[n], cols[a] (typed as above), nulls[a] may be NULL */
int sdg_push(sdg_engine* e, int stream, int64_t n, const int64_t* ts, const void* const* cols,
             const uint8_t* const* nulls);
/* InputHandler.send(Event[]) (core/stream/input/InputHandler.java:85-95): the same columns as sdg_push, but a
 * playback app's clock first moves to the LAST event's timestamp (absent-state timers due by then fire before the
 * first event) and the events themselves do not move it; sdg_push is a sequence of send(long, Object[]) calls */
int sdg_push_events(sdg_engine* e, int stream, int64_t n, const int64_t* ts, const void* const* cols,
                    const uint8_t* const* nulls);
/* rows of several streams in one interleaved batch (InputHandler.send calls of different streams, in order):
 * row i belongs to stream streams[i]; attribute a of that row is slots[a][i] as a 64-bit slot (INT/LONG the value,
 * FLOAT/DOUBLE the bit pattern in the low bits, BOOL 0/1, STRING an sdg_intern id); nulls[a] optional */
int sdg_push_mixed(sdg_engine* e, int64_t n, const int32_t* streams, const int64_t* ts, int32_t n_attrs,
                   const int64_t* const* slots, const uint8_t* const* nulls);
/* the same with device-resident columns (no copy; the caller keeps them alive until sdg_flush returns). Partition
 * keys: string attributes as sdg_intern ids; int / long attributes as their values (mapped to key ids on the device,
 * ValuePartitionExecutor.java:34-40 toString semantics); no null keys, no range partitions */
int sdg_push_device(sdg_engine* e, int stream, int64_t n, const int64_t* d_ts, const void* const* d_cols,
                    const uint8_t* const* d_nulls);
/* the clock moves to ts (playback: TimestampGeneratorImpl.setCurrentTimestamp when ts >= clock; live: the wall
 * clock reached ts). It is a position in the next flush: absent-state timers due by then fire there, before the
 * events pushed after it (Scheduler.java:71-103) */
int sdg_advance_time(sdg_engine* e, int64_t ts);
/* SiddhiAppRuntime.start(): live (non-playback) apps start their clock at ts; before any push */
int sdg_start(sdg_engine* e, int64_t ts);
/* events buffered since the last flush (a push that reaches batch_capacity flushes: the count drops) */
int64_t sdg_pending(sdg_engine* e);
int sdg_flush(sdg_engine* e);
int sdg_sync(sdg_engine* e);
int sdg_poll(sdg_engine* e, int query, sdg_out* out);
/* a multi-value selection (`e1.price` of a count state e1 without [index]: MultiValueVariableFunctionExecutor,
 * ExpressionParser.java:1430-1436) in the last sdg_poll: values[attr][i] is record i's list length; its elements are
 * items[0..cap)[i] / item_nulls[0..cap)[i] (elements past the length are null), typed *elem_type. *cap = 0: attr is
 * not a list. Valid until the next sdg_poll. */
int sdg_poll_list(sdg_engine* e, int query, int attr, int32_t* cap, int32_t* elem_type, const int64_t* const** items,
                  const uint8_t* const** item_nulls);
/* drop every query's unpolled results without reading them back (measurement of the device-resident path; an
 * application that wants its matches polls instead) */
int sdg_discard(sdg_engine* e);
/* device-side export of query `query`'s records from the last flush (instead of sdg_poll), for a multi-GPU ordered
 * gather: copied device-to-device, unordered, into caller buffers of `cap` records (d_vals: [n_out][cap]); the
 * delivery order is (event_seq, sub) ascending -- event_seq = position of the emitting event, sub = the ordinal
 * within it (chain path: the e1 event's position). *n_out = the record count. A null d_ts / d_seq / d_sub / d_vals
 * is not exported (a gather keyed on output attributes needs neither position column). Not for queries with absent
 * states (their timer matches are ordered on the host). */
int sdg_export_device(sdg_engine* e, int query, int64_t cap, int64_t* n_out, int64_t* d_ts, int64_t* d_seq,
                      int64_t* d_sub, int64_t* d_vals);
/* sdg_export_device with the records already in delivery order ((event_seq, sub) ascending, put in order on the
 * device by the same pass sdg_poll uses): each rank's export is a sorted run, so a multi-GPU gather only merges */
int sdg_export_ordered(sdg_engine* e, int query, int64_t cap, int64_t* n_out, int64_t* d_ts, int64_t* d_seq,
                       int64_t* d_sub, int64_t* d_vals);

/* SiddhiAppRuntime.snapshot() / restore(byte[]) (core/SiddhiAppRuntimeImpl.java:677-737): every partial match,
 * carried partial, timer queue, aggregator and key dictionary of the engine, after flushing what was pushed. The
 * bytes stay valid until the next sdg_snapshot / sdg_destroy. sdg_restore takes a snapshot of an engine compiled
 * from the same app text (else SDG_ERR_ARG, CannotRestoreSiddhiAppStateException) and nothing pending. */
int sdg_snapshot(sdg_engine* e, const uint8_t** data, int64_t* len);
int sdg_restore(sdg_engine* e, const uint8_t* data, int64_t len);
/* a snapshot of this app decoded into the reference's state maps: per query, per partition key, per processor the
 * StreamPreState.snapshot() map (core/query/input/stream/state/StreamPreStateProcessor.java:450-459, + the Count /
 * Absent / AbsentLogical fields), as JSON (layout in DESIGN.md "Snapshot state maps"). Needs no device: the blob
 * holds the arenas. The text stays valid until the next call / sdg_destroy. */
int sdg_snapshot_states(sdg_engine* e, const uint8_t* data, int64_t len, const char** json, int64_t* json_len);

/* introspection for measurement: device time of the last flush per kernel family, algorithmic bytes,
 * match count, and which kernel path each query took (0 = chain, 1 = generic). */
typedef struct sdg_stats {
    int64_t events;            /* events processed by the last flush (all queries) */
    int64_t matches;           /* output events produced by the last flush */
    double ms_keygroup;        /* device ms: key grouping (histogram + scan + scatter) */
    double ms_match;           /* device ms: NFA / match kernels */
    double ms_total;           /* device ms: whole flush */
    int64_t keygroup_launches;
    int64_t match_launches;
    int32_t path;              /* 0 chain (independent partials), 1 generic keyed NFA, 2 register sequence kernel */
    int32_t overflow;          /* capacity overflows detected (0 on a valid run) */
    /* device ms per kernel (HIP events on the engine's stream), summed over the flush's queries */
    double ms_kg_hist, ms_kg_prefix, ms_kg_scatter, ms_chain_carry, ms_chain_match;
    double ms_nfa;             /* generic keyed-NFA kernel */
    double ms_chain_emit;      /* chain path: match-record emission (ms_chain_match is then the deque pass) */
    int32_t deque;             /* chain path took the deque kernel (1 stack, 2 complete-all), 0 forward scans */
    int32_t fused;             /* chain path: 1 fused bucket matcher, 2 tried it and fell back to the radix path */
    int64_t fused_ovf;         /* fused path: partials resolved by the key-filtered bucket scan in HBM */
    int64_t sched_fires;       /* absent-state timer fires (Scheduler.sendTimerEvents) in the last flush */
    int64_t sched_shifted;     /* fires the reference's scheduler ran later than the key's device run did (same
                                  result, later in the delivery order) */
    int64_t sched_host_keys;   /* keys the scheduler simulation replayed on the host (their order changed results) */
    int64_t sched_rerun_keys;  /* keys rerun on the device with the scheduler's fire order (optimistic pass) */
    double ms_nfa_kernel;      /* device ms inside nfa_k launches (first run + reruns); ms_nfa also counts the host
                                  scheduler simulation, log read-back and host replays between them */
    double ms_sched_host;      /* host ms: scheduler simulation passes, log read-back, host replays */
    int64_t arena_growths;     /* generic NFA: times a key ran out of partial-match slots and the arenas doubled
                                  (the batch reran from its start; max_partials is the starting size, 4096 the
                                  device cap -- a key past it spills to the host, spilled_keys) */
    int64_t carry_in;          /* chain path: partials carried into the last flush from the one before */
    int64_t carry_out;         /* chain path: partials the last flush carries into the next */
    int64_t arena_slots;       /* generic NFA: per-key arenas allocated after the last flush (queries summed); keys
                                  whose state the reference destroys down to their start seeds give theirs back */
    int64_t sched_exact_passes; /* scheduler simulation: exact passes run (0 when the device reruns reproduced the
                                   optimistic pass's model changes, SchedSim::confirm) */
    int32_t sorted_view;       /* chain path: 1 the LDS-staged sorted-view matcher ran (carried partials folded into
                                  the key sort), 0 otherwise */
    int32_t spilled_keys;      /* generic NFA: partition keys the last flush moved to the host because they outgrew
                                  the device arena's 4096 partial matches (they run there from then on) */
    int64_t host_rows;         /* rows of the last flush processed on the host (the engine's NFA code, not the test
                                  oracle): spilled keys' rows plus the scheduler's host replays (sched_host_keys) */
    int32_t sub_batches;       /* fused chain path: time sub-batches the last flush ran in (0 / 1: the whole batch at once;
                                  SDG_FU_SUB) */
} sdg_stats;
int sdg_last_stats(sdg_engine* e, sdg_stats* out);

/* The ordered result gather's merge on rank 0 (one ordered delivery per input event,
 * core/query/input/StateMultiProcessStreamReceiver.java:47-68 and core/stream/output/StreamCallback.java:93-129): the
 * G <= 32 ranks' exports are runs already sorted by their int64 key (sdg_export_ordered), merged on the device into
 * (key, run, index in run) order -- a stable G-way merge, no re-sort. All pointers are device memory of `device`:
 * keys[r] (lens[r] records, non-decreasing), cols[r * ncols + c] (ncols <= 16 payload columns of widths[c] = 1, 2, 4
 * or 8 bytes), out_keys / out_cols[c] (sum of lens records). Synchronous: returns when the outputs are written. */
int sdg_merge_runs(int32_t device, int32_t G, const int64_t* const* keys, const int64_t* lens, int32_t ncols,
                   const void* const* cols, const uint8_t* widths, int64_t* out_keys, void* const* out_cols);

#ifdef __cplusplus
}
#endif
#endif
