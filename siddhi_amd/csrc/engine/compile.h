// Host-side query compiler: SiddhiQL AST -> sdg::Plan (NFA table + condition bytecode).
#pragma once
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <vector>

#include "../siddhiql/ast.h"
#include "plan.h"

namespace sdg {

struct Interner {
    std::unordered_map<std::string, uint32_t> ids;
    std::vector<std::string> strs;
    uint32_t get(const std::string& s) {
        auto it = ids.find(s);
        if (it != ids.end()) return it->second;
        uint32_t id = (uint32_t)strs.size();
        strs.push_back(s);
        ids.emplace(s, id);
        return id;
    }
};

struct CompileError : std::runtime_error {
    int code;  // sdg_status
    CompileError(int c, const std::string& m) : std::runtime_error(m), code(c) {}
};

struct HostQuery {
    std::string name, target;
    int partition = -1;
    Plan plan;
    std::vector<Instr> code;
    std::vector<int64_t> consts;
    std::vector<int> streams;                          // app stream index, receiver (first appearance) order
    std::vector<std::pair<std::string, uint8_t>> cols; // physical column (attribute name, kind)
    std::vector<std::vector<int>> col_attr;            // [query stream][column] -> attribute index or -1
    std::vector<int> key_attr;                         // [query stream] partition key attribute (-1: none, -2: ranges,
                                                       //  -3: no key in the partition: broadcast to every key)
    struct RangeKey {
        Prog cond;                                     // over the stream's event (OP_LOAD slot 0, physical columns)
        uint32_t label;                                // interned label: the partition key when cond holds
    };
    std::vector<std::vector<RangeKey>> key_ranges;     // [query stream] range partition executors, in order
    std::vector<uint8_t> key_kind;                     // [query stream] kind of that attribute
    std::vector<std::string> out_names;
    std::vector<int32_t> out_types;
    std::vector<int> expire_order;                     // allStateProcessors order (state ids)
    std::string chain_reason;                          // why the chain fast path does / does not apply
    int stream_pos(int app_stream) const {
        for (size_t i = 0; i < streams.size(); ++i)
            if (streams[i] == app_stream) return (int)i;
        return -1;
    }
};

// compile every query of the app; throws CompileError
std::vector<HostQuery> compile_app(const sql::App& app, Interner& strings);

}  // namespace sdg
