// Recursive-descent parser for the SiddhiQL subset on the pattern/sequence path.
//
// Grammar followed: modules/siddhi-query-compiler/src/main/antlr4/io/siddhi/query/compiler/SiddhiQL.g4
//   siddhi_app / definition_stream / partition            g4:29-52, 146-163
//   query / query_section / query_output                   g4:165-172, 379-405
//   pattern_stream / every_pattern_source_chain / ...      g4:200-302
//   sequence_stream / sequence_source_chain / collect      g4:304-340, 557-562
//   math_operation precedence (alternative order)          g4:431-446
//   attribute_reference / attribute_index                  g4:461-470
// AST construction follows the visitor (qc/internal/SiddhiQLBaseVisitorImpl.java:760-1407, 2211-2447):
//   `->` and `,` chains are left-nested NextStateElements; `every` binds to the pattern_source (or the
//   parenthesised chain) right after it; `not A and B`, `B and not A` and `B or not A for t` put the absent
//   element FIRST (State.logicalNotAnd / logicalOr argument order, visitor :1000-1021);
//   `x is null` is a stream null-check iff x names a reference already seen in the query text (visitor :2223).
// Anything outside the subset raises ParseError / Unsupported with the reference's exception class name.
#pragma once
#include <cctype>
#include <cstdlib>
#include <set>
#include <stdexcept>
#include <string>
#include <vector>

#include "ast.h"

namespace sql {

struct ParseError : std::runtime_error {
    using std::runtime_error::runtime_error;
};
struct Unsupported : std::runtime_error {
    using std::runtime_error::runtime_error;
};

enum class Tok : uint8_t { ID, QID, INT, LONG, FLOAT, DOUBLE, STR, SYM, END };

struct Token {
    Tok kind;
    std::string text;  // identifier text / literal text (no suffix, no quotes) / symbol
    size_t pos;
};

inline std::string lower(const std::string& s) {
    std::string r = s;
    for (auto& c : r) c = (char)std::tolower((unsigned char)c);
    return r;
}

inline std::vector<Token> lex(const std::string& src) {
    std::vector<Token> out;
    size_t i = 0, n = src.size();
    while (i < n) {
        char c = src[i];
        if (std::isspace((unsigned char)c)) { ++i; continue; }
        if (c == '-' && i + 1 < n && src[i + 1] == '-') {  // SINGLE_LINE_COMMENT g4:863
            while (i < n && src[i] != '\n' && src[i] != '\r') ++i;
            continue;
        }
        if (c == '/' && i + 1 < n && src[i + 1] == '*') {  // MULTILINE_COMMENT g4:867
            size_t e = src.find("*/", i + 2);
            i = (e == std::string::npos) ? n : e + 2;
            continue;
        }
        size_t st = i;
        if (std::isalpha((unsigned char)c) || c == '_') {
            while (i < n && (std::isalnum((unsigned char)src[i]) || src[i] == '_')) ++i;
            out.push_back({Tok::ID, src.substr(st, i - st), st});
            continue;
        }
        if (c == '`') {
            size_t e = src.find('`', i + 1);
            if (e == std::string::npos) throw ParseError("unterminated quoted identifier");
            out.push_back({Tok::QID, src.substr(i + 1, e - i - 1), st});
            i = e + 1;
            continue;
        }
        if (c == '\'' || c == '"') {
            size_t e = src.find(c, i + 1);
            if (e == std::string::npos) throw ParseError("unterminated string literal");
            out.push_back({Tok::STR, src.substr(i + 1, e - i - 1), st});
            i = e + 1;
            continue;
        }
        bool starts_num = std::isdigit((unsigned char)c) ||
                          (c == '.' && i + 1 < n && std::isdigit((unsigned char)src[i + 1]));
        if (starts_num) {
            // INT_LITERAL / LONG_LITERAL / FLOAT_LITERAL / DOUBLE_LITERAL (g4 lexer rules)
            bool is_real = false;
            while (i < n && std::isdigit((unsigned char)src[i])) ++i;
            if (i < n && src[i] == '.' && !(i + 1 < n && src[i + 1] == '.')) {
                // a '.' followed by an identifier start is an attribute access on a number -> not part of it
                if (!(i + 1 < n && std::isalpha((unsigned char)src[i + 1]) &&
                      std::tolower((unsigned char)src[i + 1]) != 'e' && std::tolower((unsigned char)src[i + 1]) != 'f' &&
                      std::tolower((unsigned char)src[i + 1]) != 'd')) {
                    is_real = true;
                    ++i;
                    while (i < n && std::isdigit((unsigned char)src[i])) ++i;
                }
            }
            if (i < n && (src[i] == 'e' || src[i] == 'E')) {
                size_t j = i + 1;
                if (j < n && (src[j] == '+' || src[j] == '-')) ++j;
                if (j < n && std::isdigit((unsigned char)src[j])) {
                    is_real = true;
                    i = j;
                    while (i < n && std::isdigit((unsigned char)src[i])) ++i;
                }
            }
            std::string num = src.substr(st, i - st);
            Tok k = is_real ? Tok::DOUBLE : Tok::INT;
            if (i < n) {
                char s = (char)std::tolower((unsigned char)src[i]);
                bool next_ident = i + 1 < n && (std::isalnum((unsigned char)src[i + 1]) || src[i + 1] == '_');
                if (!next_ident) {
                    if (s == 'l' && !is_real) { k = Tok::LONG; ++i; }
                    else if (s == 'f') { k = Tok::FLOAT; ++i; }
                    else if (s == 'd') { k = Tok::DOUBLE; ++i; }
                }
            }
            out.push_back({k, num, st});
            continue;
        }
        static const char* two[] = {"->", "==", "!=", ">=", "<=", nullptr};
        bool matched = false;
        for (int t = 0; two[t]; ++t) {
            if (src.compare(i, 2, two[t]) == 0) {
                out.push_back({Tok::SYM, two[t], st});
                i += 2;
                matched = true;
                break;
            }
        }
        if (matched) continue;
        if (std::string("()[],;:.=<>+-*/%@#!?").find(c) != std::string::npos) {
            out.push_back({Tok::SYM, std::string(1, c), st});
            ++i;
            continue;
        }
        throw ParseError(std::string("unexpected character '") + c + "' at " + std::to_string(i));
    }
    out.push_back({Tok::END, "", n});
    return out;
}

class Parser {
   public:
    explicit Parser(const std::string& src) : t_(lex(src)) {}

    App parse_app() {
        App app;
        std::vector<Ann> pending;
        int qcount = 0;
        while (!at_end()) {
            if (sym(";")) { ++p_; continue; }
            if (sym("@")) {
                Ann a = parse_annotation();
                if (lower(a.ns) == "app") {
                    std::string nm = lower(a.name);
                    if (nm == "name") app.name = a.first_value();
                    else if (nm == "playback") app.playback = true;
                    // @app:statistics / @app:description etc.: no role on the path
                } else {
                    pending.push_back(a);
                }
                continue;
            }
            if (kw("define")) {
                ++p_;
                if (!kw("stream")) throw Unsupported("only 'define stream' is supported on the pattern path");
                ++p_;
                app.streams.push_back(parse_stream_def());
                check_definition_annotations(pending);
                pending.clear();
                continue;
            }
            if (kw("from")) {
                Query q = parse_query(pending, qcount);
                pending.clear();
                app.queries.push_back(std::move(q));
                continue;
            }
            if (kw("partition")) {
                parse_partition(app, pending, qcount);
                pending.clear();
                continue;
            }
            throw ParseError("unexpected token '" + cur().text + "' at " + std::to_string(cur().pos));
        }
        return app;
    }

   private:
    struct Ann {
        std::string ns, name;
        std::vector<std::pair<std::string, std::string>> elems;
        std::string first_value() const { return elems.empty() ? "" : elems[0].second; }
        std::string get(const std::string& k) const {
            for (auto& e : elems)
                if (lower(e.first) == k) return e.second;
            return "";
        }
    };

    std::vector<Token> t_;
    size_t p_ = 0;
    std::set<std::string> refs_seen_;  // activeStreams of the visitor

    const Token& cur() const { return t_[p_]; }
    const Token& peek(int k = 1) const { return t_[std::min(p_ + k, t_.size() - 1)]; }
    bool at_end() const { return cur().kind == Tok::END; }
    bool sym(const char* s) const { return cur().kind == Tok::SYM && cur().text == s; }
    bool sym_at(int k, const char* s) const { return peek(k).kind == Tok::SYM && peek(k).text == s; }
    bool kw(const char* s) const { return cur().kind == Tok::ID && lower(cur().text) == s; }
    bool kw_at(int k, const char* s) const { return peek(k).kind == Tok::ID && lower(peek(k).text) == s; }
    void expect_sym(const char* s) {
        if (!sym(s)) throw ParseError(std::string("expected '") + s + "' but found '" + cur().text + "' at " + std::to_string(cur().pos));
        ++p_;
    }
    void expect_kw(const char* s) {
        if (!kw(s)) throw ParseError(std::string("expected '") + s + "' but found '" + cur().text + "' at " + std::to_string(cur().pos));
        ++p_;
    }
    std::string name() {
        if (cur().kind != Tok::ID && cur().kind != Tok::QID)
            throw ParseError("expected a name but found '" + cur().text + "' at " + std::to_string(cur().pos));
        return t_[p_++].text;
    }

    Ann parse_annotation() {
        expect_sym("@");
        Ann a;
        a.name = name();
        if (sym(":")) {
            ++p_;
            a.ns = a.name;
            a.name = name();
        }
        if (sym("(")) {
            ++p_;
            while (!sym(")")) {
                if (sym("@")) {  // nested annotation: ignored
                    parse_annotation();
                } else {
                    std::string key, val;
                    if (cur().kind == Tok::STR && !sym_at(1, "=")) {
                        val = t_[p_++].text;
                    } else {
                        if (cur().kind == Tok::STR) key = t_[p_++].text;
                        else {
                            key = name();
                            while (sym(".") || sym("-") || sym(":")) { key += t_[p_++].text; key += name(); }
                        }
                        expect_sym("=");
                        if (cur().kind != Tok::STR) throw ParseError("annotation value must be a string");
                        val = t_[p_++].text;
                    }
                    a.elems.push_back({key, val});
                }
                if (sym(",")) ++p_;
                else break;
            }
            expect_sym(")");
        }
        return a;
    }

    void check_definition_annotations(const std::vector<Ann>& anns) {
        for (auto& a : anns) {
            std::string n = lower(a.name);
            // @Async(buffer.size, workers, batch.size.max): StreamJunction hands events to a disruptor ring
            // (StreamJunction.java:101-131, 276-305) -- same per-stream order, consumed on another thread. The engine
            // consumes every pushed event in push order at its flush, which is one valid schedule of that
            // asynchronous hand-off, so the annotation is accepted and has no further effect.
            if (n == "async") continue;
            if (n == "source" || n == "sink" || n == "store" || n == "onerror")
                throw Unsupported("@" + a.name + " on a stream definition is not supported by the pattern engine");
        }
    }

    static Type parse_type(const std::string& s) {
        std::string l = lower(s);
        if (l == "int") return Type::INT;
        if (l == "long") return Type::LONG;
        if (l == "float") return Type::FLOAT;
        if (l == "double") return Type::DOUBLE;
        if (l == "bool") return Type::BOOL;
        if (l == "string") return Type::STRING;
        if (l == "object") return Type::OBJECT;
        throw ParseError("unknown attribute type '" + s + "'");
    }

    StreamDefinition parse_stream_def() {
        StreamDefinition d;
        if (sym("#") || sym("!")) throw Unsupported("inner/fault stream definitions are not supported");
        d.id = name();
        expect_sym("(");
        while (true) {
            Attribute a;
            a.name = name();
            a.type = parse_type(name());
            d.attrs.push_back(a);
            if (sym(",")) { ++p_; continue; }
            break;
        }
        expect_sym(")");
        return d;
    }

    void parse_partition(App& app, std::vector<Ann>& pending, int& qcount) {
        expect_kw("partition");
        expect_kw("with");
        expect_sym("(");
        Partition part;
        int pidx = (int)app.partitions.size();
        while (true) {
            PartitionWith w;
            ExprP first = parse_expr();
            if (kw("as")) {  // condition_ranges: condition_range (or condition_range)*, condition_range: expr as 'label'
                auto range = [&](ExprP cond) {
                    expect_kw("as");
                    if (cur().kind != Tok::STR) throw ParseError("range partition label must be a string at " + std::to_string(cur().pos));
                    w.ranges.push_back({cond, t_[p_++].text});
                };
                range(first);
                while (kw("or")) {
                    ++p_;
                    range(parse_expr());
                }
            } else {
                w.expr = first;
            }
            expect_kw("of");
            w.stream_id = name();
            part.with.push_back(w);
            if (sym(",")) { ++p_; continue; }
            break;
        }
        expect_sym(")");
        expect_kw("begin");
        std::vector<Ann> qanns;
        while (!kw("end")) {
            if (sym(";")) { ++p_; continue; }
            if (sym("@")) { qanns.push_back(parse_annotation()); continue; }
            if (!kw("from")) throw ParseError("expected a query inside partition at " + std::to_string(cur().pos));
            Query q = parse_query(qanns, qcount);
            qanns.clear();
            q.partition_index = pidx;
            part.queries.push_back((int)app.queries.size());
            app.queries.push_back(std::move(q));
        }
        expect_kw("end");
        for (auto& a : pending) {  // PartitionRuntimeImpl constructor :120-150
            if (lower(a.name) != "purge") continue;
            const std::string en = lower(a.get("enable"));
            if (en.empty()) throw ParseError("Annotation @purge is missing element 'enable'");
            if (en != "true" && en != "false") throw ParseError("Invalid value for enable: " + en + ". Please use 'true' or 'false'");
            part.purge = en == "true";
            const std::string idle = a.get("idle.period");
            if (idle.empty()) throw ParseError("Annotation @purge is missing element 'idle.period'");
            part.purge_idle_ms = annotation_time(idle);
            const std::string iv = a.get("interval");
            if (!iv.empty()) part.purge_interval_ms = annotation_time(iv);
        }
        app.partitions.push_back(part);
    }

    Query parse_query(const std::vector<Ann>& anns, int& qcount) {
        Query q;
        for (auto& a : anns) {
            std::string n = lower(a.name);
            if (n == "info") q.name = a.get("name");
            else if (n == "synchronized") { /* serialisation is inherent per handle */ }
            else if (n == "dist" || n == "async") throw Unsupported("@" + a.name + " on a query is not supported");
        }
        if (q.name.empty()) q.name = "query_" + std::to_string(qcount);
        ++qcount;
        refs_seen_.clear();
        expect_kw("from");
        parse_state_input(q);
        if (kw("select")) {
            ++p_;
            if (sym("*")) { ++p_; q.select_all = true; }
            else {
                while (true) {
                    OutputAttribute oa;
                    size_t st = p_;
                    oa.expr = parse_expr();
                    if (kw("as")) { ++p_; oa.rename = name(); }
                    else {
                        if (oa.expr->kind != ExprKind::VAR)
                            throw ParseError("output attribute at " + std::to_string(t_[st].pos) + " needs an 'as' name");
                        oa.rename = oa.expr->attr;
                    }
                    q.select.push_back(oa);
                    if (sym(",")) { ++p_; continue; }
                    break;
                }
            }
            if (kw("group")) throw Unsupported("group by is out of scope on the pattern path");
            if (kw("having")) {
                ++p_;
                q.having = parse_expr();
            }
            if (kw("order") || kw("limit") || kw("offset"))
                throw Unsupported("order by / limit / offset are out of scope on the pattern path");
        } else {
            q.select_all = true;
        }
        if (kw("output")) throw Unsupported("output rate limiting is out of scope (pass-through only)");
        if (kw("insert")) {
            ++p_;
            if (kw("current") || kw("expired") || kw("all")) {
                std::string k = lower(t_[p_++].text);
                q.out_type = k == "current" ? OutputEventType::CURRENT : k == "expired" ? OutputEventType::EXPIRED : OutputEventType::ALL;
                expect_kw("events");
            } else if (kw("events")) {
                ++p_;
            }
            expect_kw("into");
            if (sym("#")) { ++p_; q.target_inner = true; }
            q.target = name();
        } else if (kw("return")) {
            throw Unsupported("'return' queries are only valid inside anonymous streams");
        } else {
            throw Unsupported("only 'insert into' outputs are supported on the pattern path");
        }
        return q;
    }

    // ---- state input ----------------------------------------------------------------------------
    // Separator of the top-level chain decides PATTERN ('->') vs SEQUENCE (',').
    void parse_state_input(Query& q) {
        int sep = 0;  // 0 unknown, 1 pattern, 2 sequence
        bool stateful_marker = false;
        StateP root = parse_chain(sep, stateful_marker);
        if (sep == 0 && !stateful_marker)
            throw Unsupported("plain stream queries (no pattern/sequence) are not on the accelerated path");
        q.state_type = (sep == 2) ? StateType::SEQUENCE : StateType::PATTERN;
        q.root = root;
        if (kw("within")) {
            ++p_;
            q.has_within = true;
            q.within_ms = parse_time_value();
        }
    }

    StateP parse_chain(int& sep, bool& marker) {
        StateP left = parse_term(sep, marker);
        while (sym("->") || sym(",")) {
            int s = sym("->") ? 1 : 2;
            if (sep != 0 && sep != s) throw ParseError("cannot mix '->' and ',' in one state input");
            sep = s;
            ++p_;
            StateP right = parse_term(sep, marker);
            auto n = std::make_shared<StateElement>();
            n->kind = StateKind::NEXT;
            n->kids = {left, right};
            left = n;
        }
        return left;
    }

    StateP parse_term(int& sep, bool& marker) {
        if (kw("every")) {
            ++p_;
            marker = true;
            auto e = std::make_shared<StateElement>();
            e->kind = StateKind::EVERY;
            if (sym("(")) {
                ++p_;
                e->kids = {parse_chain(sep, marker)};
                expect_sym(")");
            } else {
                e->kids = {parse_source(marker)};
            }
            return e;
        }
        if (sym("(")) {
            ++p_;
            StateP inner = parse_chain(sep, marker);
            expect_sym(")");
            return inner;
        }
        return parse_source(marker);
    }

    // pattern_source / sequence_source (g4:246-249, 336-338) incl. logical and absent forms
    StateP parse_source(bool& marker) {
        StateP first;
        if (kw("not")) {
            marker = true;
            first = parse_absent();
        } else {
            first = parse_stateful();
            if (!first->ref.empty()) marker = true;
            // collect / quantifiers
            if (sym("<")) {
                ++p_;
                marker = true;
                auto c = std::make_shared<StateElement>();
                c->kind = StateKind::COUNT;
                c->kids = {first};
                if (sym(":")) {
                    ++p_;
                    c->max_count = parse_int();
                } else {
                    int a = parse_int();
                    if (sym(":")) {
                        ++p_;
                        c->min_count = a;
                        if (cur().kind == Tok::INT) c->max_count = parse_int();
                    } else {
                        c->min_count = a;
                        c->max_count = a;
                    }
                }
                expect_sym(">");
                return c;
            }
            if (sym("*") || sym("+") || sym("?")) {
                marker = true;
                auto c = std::make_shared<StateElement>();
                c->kind = StateKind::COUNT;
                c->kids = {first};
                std::string s = t_[p_++].text;
                if (s == "*") { c->min_count = 0; c->max_count = COUNT_ANY; }
                else if (s == "+") { c->min_count = 1; c->max_count = COUNT_ANY; }
                else { c->min_count = 0; c->max_count = 1; }
                c->seq_quantifier = true;
                return c;
            }
        }
        if (kw("and") || kw("or")) {
            marker = true;
            auto l = std::make_shared<StateElement>();
            l->kind = StateKind::LOGICAL;
            l->logical = kw("and") ? LogicalType::AND : LogicalType::OR;
            ++p_;
            StateP second;
            if (kw("not")) second = parse_absent();
            else second = parse_stateful();
            bool a1 = first->kind == StateKind::ABSENT, a2 = second->kind == StateKind::ABSENT;
            if (l->logical == LogicalType::OR && (a1 || a2) && !(a1 && a2)) {
                if (a1 && !first->has_waiting) throw ParseError("'not ... or' requires 'for <time>'");
                if (a2 && !second->has_waiting) throw ParseError("'or not ...' requires 'for <time>'");
            }
            if (a2 && !a1) l->kids = {second, first};  // State.logicalNotAnd / logicalOr(absent, present)
            else l->kids = {first, second};
            return l;
        }
        if (first->kind == StateKind::ABSENT && !first->has_waiting)
            throw ParseError("'not' pattern without 'for' must be combined with 'and'");
        return first;
    }

    StateP parse_absent() {
        expect_kw("not");
        StateP s = parse_stateful();
        if (!s->ref.empty()) throw ParseError("NOT pattern cannot have reference id but found " + s->ref);
        s->kind = StateKind::ABSENT;
        if (kw("for")) {
            ++p_;
            s->has_waiting = true;
            s->waiting_ms = parse_time_value();
        }
        return s;
    }

    StateP parse_stateful() {
        auto s = std::make_shared<StateElement>();
        s->kind = StateKind::STREAM;
        if ((cur().kind == Tok::ID || cur().kind == Tok::QID) && sym_at(1, "=")) {
            s->ref = name();
            ++p_;
        }
        if (sym("#")) { ++p_; s->inner = true; }
        else if (sym("!")) { ++p_; s->fault = true; }
        if (s->inner || s->fault) throw Unsupported("inner/fault streams are not supported on the pattern path");
        s->stream_id = name();
        while (true) {
            if (sym("[")) {
                ++p_;
                s->filters.push_back(parse_expr());
                expect_sym("]");
            } else if (sym("#") && sym_at(1, "[")) {
                p_ += 2;
                s->filters.push_back(parse_expr());
                expect_sym("]");
            } else if (sym("#")) {
                throw Unsupported("stream functions / windows inside a pattern are out of scope");
            } else {
                break;
            }
        }
        if (!s->ref.empty()) refs_seen_.insert(s->ref);
        return s;
    }

    int parse_int() {
        if (cur().kind != Tok::INT) throw ParseError("expected an integer at " + std::to_string(cur().pos));
        return std::atoi(t_[p_++].text.c_str());
    }

    static bool time_unit(const std::string& w, int64_t& mult) {
        std::string l = lower(w);
        // lexer rules g4 YEARS..MILLISECONDS; multipliers TimeConstant.java
        if (l == "year" || l == "years") { mult = 31556900000LL; return true; }
        if (l == "month" || l == "months") { mult = 2630000000LL; return true; }
        if (l == "week" || l == "weeks") { mult = 7LL * 24 * 3600 * 1000; return true; }
        if (l == "day" || l == "days") { mult = 24LL * 3600 * 1000; return true; }
        if (l == "hour" || l == "hours") { mult = 3600LL * 1000; return true; }
        if (l == "min" || l == "minute" || l == "minutes") { mult = 60LL * 1000; return true; }
        if (l == "sec" || l == "second" || l == "seconds") { mult = 1000; return true; }
        if (l == "millisec" || l == "millisecond" || l == "milliseconds") { mult = 1; return true; }
        return false;
    }

    // Expression.Time.timeToLong (siddhi-query-api .../expression/Expression.java:250-290): the first digit run and
    // the first non-digit run of an annotation value ("1 sec", "2 min")
    static int64_t annotation_time(const std::string& v) {
        size_t i = 0;
        while (i < v.size() && !std::isdigit((unsigned char)v[i])) ++i;
        size_t j = i;
        while (j < v.size() && std::isdigit((unsigned char)v[j])) ++j;
        size_t a = 0;
        while (a < v.size() && std::isdigit((unsigned char)v[a])) ++a;
        size_t b = a;
        while (b < v.size() && !std::isdigit((unsigned char)v[b])) ++b;
        std::string unit = lower(v.substr(a, b - a));
        while (!unit.empty() && std::isspace((unsigned char)unit.back())) unit.pop_back();
        while (!unit.empty() && std::isspace((unsigned char)unit.front())) unit.erase(unit.begin());
        if (i == j || unit.empty()) throw ParseError("Provided retention value cannot be identified: " + v);
        const int64_t n = std::atoll(v.substr(i, j - i).c_str());
        if (unit == "sec" || unit == "seconds" || unit == "second") return n * 1000;
        if (unit == "min" || unit == "minutes" || unit == "minute") return n * 60000;
        if (unit == "h" || unit == "hour" || unit == "hours") return n * 3600000;
        if (unit == "day" || unit == "days") return n * 86400000;
        if (unit == "year" || unit == "years") return n * 31556900000LL;
        if (unit == "month" || unit == "months") return n * 2630000000LL;
        throw ParseError("Provided retention value cannot be identified: " + v);
    }

    int64_t parse_time_value() {
        int64_t total = 0;
        bool any = false;
        int64_t m;
        while (cur().kind == Tok::INT && peek().kind == Tok::ID && time_unit(peek().text, m)) {
            total += std::atoll(cur().text.c_str()) * m;
            p_ += 2;
            any = true;
        }
        if (!any) throw ParseError("expected a time value at " + std::to_string(cur().pos));
        return total;
    }

    // ---- expressions ----------------------------------------------------------------------------
    ExprP mk(ExprKind k) {
        auto e = std::make_shared<Expr>();
        e->kind = k;
        return e;
    }
    ExprP bin(ExprKind k, ExprP a, ExprP b) {
        auto e = mk(k);
        e->kids = {a, b};
        return e;
    }

   public:
    ExprP parse_expr() { return parse_or(); }

   private:
    ExprP parse_or() {
        ExprP l = parse_and();
        while (kw("or")) { ++p_; l = bin(ExprKind::OR, l, parse_and()); }
        return l;
    }
    ExprP parse_and() {
        ExprP l = parse_eq();
        while (kw("and")) { ++p_; l = bin(ExprKind::AND, l, parse_eq()); }
        return l;
    }
    ExprP parse_eq() {
        ExprP l = parse_rel();
        if (kw("in")) throw Unsupported("'in <table>' is out of scope");
        while (sym("==") || sym("!=")) {
            auto e = mk(ExprKind::CMP);
            e->cmp = sym("==") ? CmpOp::EQ : CmpOp::NE;
            ++p_;
            e->kids = {l, parse_rel()};
            l = e;
        }
        return l;
    }
    ExprP parse_rel() {
        ExprP l = parse_add();
        while (sym(">=") || sym("<=") || sym(">") || sym("<")) {
            auto e = mk(ExprKind::CMP);
            std::string s = cur().text;
            e->cmp = s == ">=" ? CmpOp::GE : s == "<=" ? CmpOp::LE : s == ">" ? CmpOp::GT : CmpOp::LT;
            ++p_;
            e->kids = {l, parse_add()};
            l = e;
        }
        return l;
    }
    ExprP parse_add() {
        ExprP l = parse_mul();
        while (sym("+") || sym("-")) {
            ExprKind k = sym("+") ? ExprKind::ADD : ExprKind::SUB;
            ++p_;
            l = bin(k, l, parse_mul());
        }
        return l;
    }
    ExprP parse_mul() {
        ExprP l = parse_unary();
        while (sym("*") || sym("/") || sym("%")) {
            ExprKind k = sym("*") ? ExprKind::MUL : sym("/") ? ExprKind::DIV : ExprKind::MOD;
            ++p_;
            l = bin(k, l, parse_unary());
        }
        return l;
    }
    ExprP parse_unary() {
        if (kw("not")) {
            ++p_;
            auto e = mk(ExprKind::NOT);
            e->kids = {parse_unary()};
            return e;
        }
        return parse_primary();
    }

    bool is_null_next() const { return kw("is") && kw_at(1, "null"); }
    ExprP wrap_is_null(ExprP e) {
        if (is_null_next()) {
            p_ += 2;
            auto n = mk(ExprKind::IS_NULL);
            n->kids = {e};
            return n;
        }
        return e;
    }

    ExprP parse_number(bool neg) {
        const Token& t = cur();
        auto e = mk(ExprKind::CONST);
        std::string txt = (neg ? "-" : "") + t.text;
        switch (t.kind) {
            case Tok::INT: e->c.type = Type::INT; e->c.i = (int32_t)std::strtoll(txt.c_str(), nullptr, 10); break;
            case Tok::LONG: e->c.type = Type::LONG; e->c.i = std::strtoll(txt.c_str(), nullptr, 10); break;
            case Tok::FLOAT: e->c.type = Type::FLOAT; e->c.f = std::strtof(txt.c_str(), nullptr); e->c.d = e->c.f; break;
            case Tok::DOUBLE: e->c.type = Type::DOUBLE; e->c.d = std::strtod(txt.c_str(), nullptr); break;
            default: throw ParseError("expected a number");
        }
        ++p_;
        return e;
    }

    int parse_attribute_index() {
        // attribute_index : INT_LITERAL | LAST ('-' INT_LITERAL)?   (visitor :2345-2356)
        if (kw("last")) {
            ++p_;
            int idx = IDX_LAST;
            if (sym("-")) { ++p_; idx = IDX_LAST - parse_int(); }
            return idx;
        }
        return parse_int();
    }

    ExprP parse_primary() {
        if (sym("(")) {
            ++p_;
            ExprP e = parse_expr();
            expect_sym(")");
            return e;
        }
        if ((sym("-") || sym("+")) && (peek().kind == Tok::INT || peek().kind == Tok::LONG ||
                                       peek().kind == Tok::FLOAT || peek().kind == Tok::DOUBLE)) {
            bool neg = sym("-");
            ++p_;
            return parse_number(neg);
        }
        if (cur().kind == Tok::INT) {
            int64_t m;
            if (peek().kind == Tok::ID && time_unit(peek().text, m)) {
                auto e = mk(ExprKind::CONST);
                e->c.type = Type::LONG;
                e->c.i = parse_time_value();
                return e;
            }
        }
        if (cur().kind == Tok::INT || cur().kind == Tok::LONG || cur().kind == Tok::FLOAT || cur().kind == Tok::DOUBLE)
            return parse_number(false);
        if (cur().kind == Tok::STR) {
            auto e = mk(ExprKind::CONST);
            e->c.type = Type::STRING;
            e->c.s = t_[p_++].text;
            return e;
        }
        if (kw("true") || kw("false")) {
            auto e = mk(ExprKind::CONST);
            e->c.type = Type::BOOL;
            e->c.i = kw("true") ? 1 : 0;
            ++p_;
            return e;
        }
        if (kw("null")) throw Unsupported("null literal is not supported in expressions");
        bool hash = false, bang = false;
        if (sym("#")) { hash = true; ++p_; }
        else if (sym("!")) { bang = true; ++p_; }
        if (hash || bang) throw Unsupported("inner/fault stream references are out of scope");
        if (cur().kind != Tok::ID && cur().kind != Tok::QID)
            throw ParseError("unexpected token '" + cur().text + "' at " + std::to_string(cur().pos));
        // function_operation: (ns ':')? name '(' ... ')'
        if (sym_at(1, "(") || (sym_at(1, ":") && sym_at(3, "("))) {
            auto f = mk(ExprKind::FUNC);
            if (sym_at(1, ":")) { f->fn_ns = name(); ++p_; }
            f->fn_name = name();
            expect_sym("(");
            if (sym("*")) { ++p_; }
            else if (!sym(")")) {
                while (true) {
                    f->kids.push_back(parse_expr());
                    if (sym(",")) { ++p_; continue; }
                    break;
                }
            }
            expect_sym(")");
            return wrap_is_null(f);
        }
        std::string n1 = name();
        bool has_idx = false;
        int idx = 0;
        if (sym("[")) {
            ++p_;
            has_idx = true;
            idx = parse_attribute_index();
            expect_sym("]");
        }
        if (sym("#")) throw Unsupported("'#' stream reference chains are out of scope");
        if (sym(".")) {
            ++p_;
            auto v = mk(ExprKind::VAR);
            v->stream_ref = n1;
            v->has_index = has_idx;
            v->index = idx;
            v->attr = name();
            return wrap_is_null(v);
        }
        if (is_null_next()) {
            // null_check: stream_reference first (visitor :2214-2239)
            p_ += 2;
            if (refs_seen_.count(n1)) {
                auto s = mk(ExprKind::IS_NULL_STREAM);
                s->stream_ref = n1;
                s->has_index = has_idx;
                s->index = idx;
                return s;
            }
            auto v = mk(ExprKind::VAR);
            v->attr = n1;
            auto nn = mk(ExprKind::IS_NULL);
            nn->kids = {v};
            return nn;
        }
        if (has_idx) throw ParseError("indexed reference '" + n1 + "[..]' needs an attribute");
        auto v = mk(ExprKind::VAR);
        v->attr = n1;
        return v;
    }
};

inline App parse_app(const std::string& src) {
    Parser p(src);
    return p.parse_app();
}

}  // namespace sql
