// SiddhiQL subset AST — the front end shared by the engine compiler and the oracle.
//
// Mirrors the query-api types the pattern/sequence path consumes:
//   StateInputStream / StateElement tree
//     (modules/siddhi-query-api/src/main/java/io/siddhi/query/api/execution/query/input/state/*.java)
//   Expression tree (.../query/api/expression/*.java)
// Only the subset reachable from `from <pattern|sequence> select ... insert into ...` is represented.
#pragma once
#include <cstdint>
#include <memory>
#include <string>
#include <vector>

namespace sql {

// Attribute.Type (modules/siddhi-query-api/.../definition/Attribute.java)
enum class Type : uint8_t { INT = 0, LONG = 1, FLOAT = 2, DOUBLE = 3, BOOL = 4, STRING = 5, OBJECT = 6 };

inline const char* type_name(Type t) {
    switch (t) {
        case Type::INT: return "int";
        case Type::LONG: return "long";
        case Type::FLOAT: return "float";
        case Type::DOUBLE: return "double";
        case Type::BOOL: return "bool";
        case Type::STRING: return "string";
        default: return "object";
    }
}
inline bool is_numeric(Type t) { return t <= Type::DOUBLE; }

struct Attribute {
    std::string name;
    Type type;
};

struct StreamDefinition {
    std::string id;
    std::vector<Attribute> attrs;
    int index_of(const std::string& n) const {
        for (size_t i = 0; i < attrs.size(); ++i)
            if (attrs[i].name == n) return (int)i;
        return -1;
    }
};

// A literal. Strings keep their text; the runtime interns them.
struct Constant {
    Type type = Type::INT;
    bool is_null = false;
    int64_t i = 0;  // INT / LONG / BOOL
    double d = 0;   // DOUBLE; FLOAT stored as the float's exact double value
    float f = 0;    // FLOAT
    std::string s;  // STRING
};

// SiddhiConstants.CURRENT / LAST (core/util/SiddhiConstants.java:90-91)
constexpr int IDX_CURRENT = -1;
constexpr int IDX_LAST = -2;

enum class ExprKind : uint8_t {
    CONST,
    VAR,          // [ref['['idx']'] '.'] attr
    AND, OR, NOT,
    CMP,          // op in CmpOp
    ADD, SUB, MUL, DIV, MOD,
    IS_NULL,      // <expr> is null
    IS_NULL_STREAM,  // e1 is null / e1[2] is null
    FUNC,         // function call: ifThenElse / coalesce / default / instanceOf* / maximum / minimum, aggregators
};
enum class CmpOp : uint8_t { EQ, NE, GT, GE, LT, LE };

struct Expr {
    ExprKind kind;
    CmpOp cmp = CmpOp::EQ;
    Constant c;
    // VAR / IS_NULL_STREAM
    std::string stream_ref;     // e1 / Stream1 / "" (unqualified)
    bool has_index = false;     // e1[k]
    int index = 0;              // k >= 0, or IDX_LAST - m for `last - m` (visitor: qc/internal/SiddhiQLBaseVisitorImpl.java:2345-2356)
    std::string attr;
    // FUNC
    std::string fn_ns, fn_name;
    std::vector<std::shared_ptr<Expr>> kids;
};
using ExprP = std::shared_ptr<Expr>;

// StateElement kinds (query-api .../input/state/)
enum class StateKind : uint8_t { STREAM, ABSENT, NEXT, EVERY, LOGICAL, COUNT };
enum class LogicalType : uint8_t { AND, OR };

// ANY (SiddhiConstants.ANY = -1) for open count bounds
constexpr int COUNT_ANY = -1;

struct StateElement {
    StateKind kind;
    // STREAM / ABSENT: the BasicSingleInputStream
    std::string stream_id;
    std::string ref;                  // `e1=` reference id; empty if none
    bool inner = false, fault = false;
    std::vector<ExprP> filters;       // one FilterProcessor per [..]
    bool has_waiting = false;         // ABSENT: `for <time>` present
    int64_t waiting_ms = -1;
    // COUNT
    int min_count = COUNT_ANY, max_count = COUNT_ANY;
    bool seq_quantifier = false;      // `*` `+` `?` (sequence_collection_stateful_source only)
    // LOGICAL
    LogicalType logical = LogicalType::AND;
    // NEXT: kids[0] -> kids[1]; EVERY: kids[0]; LOGICAL: kids[0] op kids[1]; COUNT: kids[0] (a STREAM)
    std::vector<std::shared_ptr<StateElement>> kids;
};
using StateP = std::shared_ptr<StateElement>;

enum class StateType : uint8_t { PATTERN, SEQUENCE };
enum class OutputEventType : uint8_t { CURRENT, EXPIRED, ALL };

struct OutputAttribute {
    std::string rename;  // `as` name (or the attribute name)
    ExprP expr;
};

struct Query {
    std::string name;           // @info(name=...) or generated
    StateType state_type = StateType::PATTERN;
    StateP root;
    bool has_within = false;
    int64_t within_ms = 0;
    bool select_all = false;
    std::vector<OutputAttribute> select;
    ExprP having;               // `having <expr>` (QuerySelector.havingConditionExecutor) or null
    std::string target;         // insert into <target>
    bool target_inner = false;
    OutputEventType out_type = OutputEventType::CURRENT;
    int partition_index = -1;   // index into App::partitions, -1 if top level
};

struct PartitionWith {
    ExprP expr;                 // value partition expression (null for a range partition)
    std::string stream_id;
    // range partition `c1 as 'l1' or c2 as 'l2' of S` (RangePartitionType): one RangePartitionExecutor per range,
    // each sends the event to partition key `label` when its condition holds (an event may go to several keys)
    std::vector<std::pair<ExprP, std::string>> ranges;
};

struct Partition {
    std::vector<PartitionWith> with;
    std::vector<int> queries;   // indices into App::queries
    // @purge(enable, interval, idle.period) (PartitionRuntimeImpl.java:120-150): idle keys' states are destroyed
    bool purge = false;
    int64_t purge_interval_ms = 300000;
    int64_t purge_idle_ms = 0;
};

struct App {
    std::string name;
    bool playback = false;
    std::vector<StreamDefinition> streams;
    std::vector<Query> queries;
    std::vector<Partition> partitions;
    const StreamDefinition* stream(const std::string& id) const {
        for (auto& s : streams)
            if (s.id == id) return &s;
        return nullptr;
    }
    int stream_index(const std::string& id) const {
        for (size_t i = 0; i < streams.size(); ++i)
            if (streams[i].id == id) return (int)i;
        return -1;
    }
};

}  // namespace sql
