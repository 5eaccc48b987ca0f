// Compiled query plan: the NFA table + condition bytecode a SiddhiQL pattern/sequence query lowers to.
// POD only: the same structs are copied verbatim into device memory and read by the kernels.
//
// Lowering contract followed (reference, paths under modules/siddhi-core/src/main/java/io/siddhi/core/):
//   state ids / start states / every / within      util/parser/StateInputStreamParser.java:76-408
//   variable positions [slot, chain index, attr]    util/parser/ExpressionParser.java:1302-1438
//   compare / arithmetic promotion, null rules      executor/condition/compare/**, executor/math/**,
//                                                   util/parser/ExpressionParser.java:568-667, 1488-1520
#pragma once
#include <stdint.h>

namespace sdg {

// value kinds == sql::Type codes 0..5 == sdg_type
enum VK : uint8_t { VK_I32 = 0, VK_I64 = 1, VK_F32 = 2, VK_F64 = 3, VK_BOOL = 4, VK_STR = 5 };

enum OpCode : uint8_t {
    OP_LOAD = 1,   // push attribute: a = state slot, b = column, c = chain index, k = kind
    OP_CONST,      // push consts[imm] (kind k)
    OP_CVT,        // convert top of stack: a = from kind, k = to kind (Number.xValue())
    OP_CMP,        // a = CmpOp, k = operand kind; pop 2, push bool; null operand -> false
    OP_ARITH,      // a = ArithOp, k = kind; pop 2, push; null propagates; int/long/float/double /,% by 0 -> null
    OP_AND,        // pop 2 push bool  (AndConditionExpressionExecutor: null -> false)
    OP_OR,         // pop 2 push bool
    OP_NOT,        // pop 1 push bool  (null -> TRUE)
    OP_ISNULL,     // pop 1 push bool
    OP_SLOTNULL,   // push bool: state slot a, chain index c is empty (IsNullStreamConditionExpressionExecutor)
    OP_COND,       // pop 1 push bool: null -> false (BoolConditionExpressionExecutor)
    OP_IFELSE,     // pop 3 (cond, then, else) push: cond non-null and true ? then : else (IfThenElseFunctionExecutor)
    OP_COALESCE,   // a = n: pop n push the first non-null one, else null (Coalesce / DefaultFunctionExecutor)
    OP_MAXMIN,     // a = n, c = 1 maximum / 0 minimum, k = kind (Maximum / MinimumFunctionExecutor)
    // selector post pass only (aggregators are stateful, so And/Or must short-circuit exactly as Java does):
    OP_AGG,        // push aggregator a's value after this record (its state updates only when this runs)
    OP_JAND,       // top not true: replace it by false and jump imm instructions ahead (past the right operand
                   // and its OP_AND); else fall through (AndConditionExpressionExecutor :65-74)
    OP_JOR,        // top true: replace it by true and jump imm ahead (OrConditionExpressionExecutor :65-76)
    OP_SLOTLEN,    // push the length of state slot a's event chain, counting at most c (a multi-value selection)
};
// OP_LOAD slot of the selector's post pass (aggregates, having): column b of the output record being selected
constexpr uint8_t OUT_SLOT = 0xFF;
enum CmpOp : uint8_t { CMP_EQ = 0, CMP_NE, CMP_GT, CMP_GE, CMP_LT, CMP_LE };
enum ArithOp : uint8_t { AR_ADD = 0, AR_SUB, AR_MUL, AR_DIV, AR_MOD };

struct Instr {
    uint8_t op, k, a, pad;
    int32_t b;     // column
    int32_t c;     // chain index (>= 0 nth; -1 CURRENT/last; -2 LAST/second to last; <= -3 from the end)
    int32_t imm;   // constant index
};

struct Prog {
    int32_t start = 0, len = 0;  // into Plan::code; len 0 == always true (no filter)
};

// A filter of the shape `a OP b` with a = attribute of a state slot and b = constant or attribute of another
// slot, recognised at compile time and evaluated natively (no interpreter); same semantics as the bytecode.
enum FastKind : uint8_t { FP_NONE = 0, FP_TRUE = 1, FP_CONST = 2, FP_SLOT = 3 };
struct FastPred {
    uint8_t kind = FP_NONE;
    uint8_t op = 0;      // CmpOp, oriented as a OP b
    uint8_t t = 0;       // comparison kind after promotion
    uint8_t ka = 0, kb = 0;
    int8_t sa = 0, sb = 0;   // state slots
    int8_t ia = -1, ib = -1; // chain indexes (count states: e1[0], e1[last] ...)
    int32_t ca = 0, cb = 0;  // columns
    int64_t konst = 0;   // FP_CONST: b already converted to kind t
};

constexpr int MAX_STATES = 16;
constexpr int MAX_OUT = 32;
constexpr int MAX_COLS = 32;
constexpr int STACK = 8;
constexpr int MAX_AGG = 8;

// attribute aggregators in a pattern query's selector (query/selector/attribute/aggregator/*), running per
// partition key over the query's output records in delivery order (the selector's post pass)
enum AggKind : uint8_t { AG_COUNT = 0, AG_SUM, AG_AVG, AG_MIN, AG_MAX };
struct AggSpec {
    uint8_t kind;       // AggKind
    uint8_t arg_kind;   // kind of the argument column
    uint8_t out_kind;   // result kind (count/sum of int,long: long; sum of float,double / avg: double; min/max: arg)
    uint8_t pad;
    int32_t arg_col;    // output-record column holding the argument (evaluated at emission), -1 for count()
    int32_t out_col;    // unused (-1): the value is pushed by OP_AGG where the expression reads it
};

// processor kinds of the generic NFA (one per PreStateProcessor)
enum ProcKind : uint8_t { PK_STREAM = 0, PK_COUNT = 1, PK_LOGICAL = 2, PK_ABSENT = 3 };

struct StateRow {
    uint8_t kind;            // ProcKind
    uint8_t is_start;
    uint8_t logical_or;      // LOGICAL: 1 = or, 0 = and
    uint8_t seq;             // SEQUENCE
    int32_t stream;          // app stream index of this state's events
    Prog filter;             // conjunction of the state's [..] filters
    int32_t next;            // nextStatePreProcessor (state id) or -1
    int32_t next_every;      // nextEveryStatePreProcessor or -1
    int32_t within_every;    // withinEveryPreStateProcessor or -1
    int32_t partner;         // LOGICAL partner state or -1
    int32_t callback;        // callbackPreStateProcessor (count) or -1
    int32_t last;            // thisLastProcessor's state id (own, or the query's last for the first state)
    int32_t min_count, max_count;
    int64_t waiting_ms;      // ABSENT / absent side of a LOGICAL (-1: no `for`)
    uint8_t selector_after;  // post.nextProcessor == selector (last state / logical partners of it)
    uint8_t absent;          // LOGICAL: this side is `not S[..]` (AbsentLogicalPreStateProcessor)
    int8_t sched;            // scheduler of this absent processor (index into Plan::sched_state) or -1
    uint8_t pad[5];
};

// per query stream: the receiver built by StateInputStreamParser (:91-110) and wired by the inner runtimes'
// setup() (query/input/stream/state/runtime/*InnerStateRuntime.java)
struct RecvRow {
    int32_t n;                   // processors subscribed to this stream (setup order)
    int32_t procs[MAX_STATES];   // nextProcessors / stateProcessorsForStream
    int32_t order[MAX_STATES];   // eventSequence (reversed for Pattern/SequenceMultiProcessStreamReceiver)
    uint8_t multi;
    uint8_t selector;            // querySelector != null
    uint8_t pad[2];
};

struct Plan {
    int32_t n_states = 0;
    int32_t seq = 0;               // SEQUENCE (1) / PATTERN (0)
    int32_t has_within = 0;
    int64_t within_ms = 0;
    int32_t partitioned = 0;
    int32_t chain = 0;             // 1: the independent-partial fast path applies
    int32_t n_out = 0;             // columns of an output record: the user's select list, then hidden columns
                                   // (aggregator arguments and results, having operands)
    int32_t n_user_out = 0;        // the select list (what sdg_poll returns)
    uint8_t out_kind[MAX_OUT];
    Prog out_prog[MAX_OUT];        // evaluated at emission (len 0: filled by the post pass)
    uint8_t out_multi[MAX_OUT];    // multi-value selection (a count state without [index]): the column holds the
                                   // list length, elements in out_list_cap hidden columns from out_list_col
    int32_t out_list_col[MAX_OUT], out_list_cap[MAX_OUT];
    int32_t n_list_cols = 0;       // hidden element columns, right after the select list
    uint8_t out_post[MAX_OUT];     // 1: a select item over aggregates, evaluated by the post pass (post_prog)
    Prog post_prog[MAX_OUT];
    int32_t n_agg = 0;
    AggSpec agg[MAX_AGG];
    Prog having;                   // post pass; len 0: no having clause
    int32_t has_post = 0;          // aggregates or having: the selector's post pass runs
    int32_t n_cols = 0;            // physical columns of this query's batch view
    uint8_t col_kind[MAX_COLS];
    int32_t n_streams = 0;         // streams this query reads, in receiver order
    int32_t streams[MAX_STATES];
    StateRow st[MAX_STATES];
    FastPred fast[MAX_STATES];     // per state filter (FP_NONE: use the bytecode)
    RecvRow recv[MAX_STATES];      // indexed by query-stream position
    int32_t n_expire, expire_seq[MAX_STATES];   // allStateProcessors (expireEvents order)
    int32_t n_init, init_seq[MAX_STATES];       // innerStateRuntime.init()
    int32_t n_reset, reset_seq[MAX_STATES];     // innerStateRuntime.reset()
    int32_t n_update, update_seq[MAX_STATES];   // innerStateRuntime.update()
    int32_t n_startup, startup_seq[MAX_STATES]; // startupPreStateProcessors (absent partitionCreated)
    int32_t n_sched, sched_state[MAX_STATES];   // one Scheduler per absent processor, in creation order (= the
                                                // order its TimeChangeListener registers, SchedulerParser.parse)
    int32_t playback;                           // @app:playback: the clock is event time (else modelled wall clock)
    int32_t purge;                              // the partition has @purge(enable='true')
    int64_t purge_interval_ms, purge_idle_ms;
    // expire order (allStateProcessors), setup order per stream etc. live on the host plan
    int32_t n_code = 0, n_consts = 0;
};

}  // namespace sdg
