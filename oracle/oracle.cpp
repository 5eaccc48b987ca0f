// Parity oracle — TEST INFRASTRUCTURE ONLY (see oracle.h). Never linked by the product.
//
// A line-by-line restatement of the reference siddhi-core pattern/sequence object model. Every class below
// names the Java file it follows (paths relative to
// /root/reference/modules/siddhi-core/src/main/java/io/siddhi/core/):
//   ComplexEventChunk            event/ComplexEventChunk.java
//   StreamEvent / StateEvent     event/stream/StreamEvent.java, event/state/StateEvent.java (+ cloners)
//   PreState / StateHolder       query/input/stream/state/StreamPreStateProcessor.java:435-498,
//                                util/snapshot/state/PartitionSyncStateHolder.java, PartitionStateHolder.java
//   PreProc / Post               query/input/stream/state/StreamPreStateProcessor.java, StreamPostStateProcessor.java
//   CountPre / CountPost         query/input/stream/state/CountPreStateProcessor.java, CountPostStateProcessor.java
//   LogicalPre / LogicalPost     query/input/stream/state/LogicalPreStateProcessor.java, LogicalPostStateProcessor.java
//   AbsentPre / AbsentPost       query/input/stream/state/AbsentStreamPreStateProcessor.java, AbsentStreamPostStateProcessor.java
//   AbsentLogicalPre / Post      query/input/stream/state/AbsentLogicalPreStateProcessor.java, AbsentLogicalPostStateProcessor.java
//   Inner runtimes               query/input/stream/state/runtime/*.java
//   Receivers                    query/input/{Single,Multi,StateMulti}ProcessStreamReceiver.java + state/receiver/*.java
//   Lowering                     util/parser/StateInputStreamParser.java:76-408
//   Executors                    executor/condition/**, executor/math/**, util/parser/ExpressionParser.java
//   Selector / outputs           query/selector/QuerySelector.java:161-205, query/output/ratelimit/OutputRateLimiter.java:64-108,
//                                query/output/callback/QueryCallback.java:60-105
//   Partition                    partition/PartitionStreamReceiver.java:150-283, partition/executor/ValuePartitionExecutor.java
//   Scheduler / clock            util/Scheduler.java:71-209,330-366, util/timestamp/TimestampGeneratorImpl.java:78-122
// Java HashMap iteration order (JDK 8 java.util.HashMap: hash spreading, computeIfAbsent head insertion,
// resize lo/hi split) is emulated for the scheduler's partition-state map, because Scheduler.onTimeChange's
// TreeMultimap collapses states whose next notify time is equal (SchedulerState.compareTo() == 0) and keeps
// the first one in that iteration order. Tree bins (>= 8 collisions in one bucket) are not emulated.
#include "oracle.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <deque>
#include <functional>
#include <list>
#include <map>
#include <set>
#include <memory>
#include <string>
#include <unordered_map>
#include <vector>

#include "../siddhi_amd/csrc/siddhiql/parser.h"

namespace orc {

using sql::Type;

struct OracleError : std::runtime_error {
    using std::runtime_error::runtime_error;
};

// ------------------------------------------------------------------------------------------------
// values (slots as in oracle.h)
struct Val {
    uint8_t t = 0;
    bool null = true;
    int64_t raw = 0;
    int32_t i() const { return (int32_t)raw; }
    int64_t l() const { return raw; }
    float f() const { uint32_t u = (uint32_t)raw; float x; std::memcpy(&x, &u, 4); return x; }
    double d() const { double x; std::memcpy(&x, &raw, 8); return x; }
    bool b() const { return raw != 0; }
};
static Val vnull(Type t) { Val v; v.t = (uint8_t)t; v.null = true; return v; }
static Val vI(int32_t x) { Val v; v.t = (uint8_t)Type::INT; v.null = false; v.raw = x; return v; }
static Val vL(int64_t x) { Val v; v.t = (uint8_t)Type::LONG; v.null = false; v.raw = x; return v; }
static Val vF(float x) { Val v; v.t = (uint8_t)Type::FLOAT; v.null = false; uint32_t u; std::memcpy(&u, &x, 4); v.raw = u; return v; }
static Val vD(double x) { Val v; v.t = (uint8_t)Type::DOUBLE; v.null = false; std::memcpy(&v.raw, &x, 8); return v; }
static Val vB(bool x) { Val v; v.t = (uint8_t)Type::BOOL; v.null = false; v.raw = x ? 1 : 0; return v; }
static Val vS(uint32_t id) { Val v; v.t = (uint8_t)Type::STRING; v.null = false; v.raw = id; return v; }

// Number.floatValue()/doubleValue()/longValue()/intValue() of a boxed numeric
static double as_double(const Val& v) {
    switch ((Type)v.t) {
        case Type::INT: return (double)v.i();
        case Type::LONG: return (double)v.l();
        case Type::FLOAT: return (double)v.f();
        default: return v.d();
    }
}
static float as_float(const Val& v) {
    switch ((Type)v.t) {
        case Type::INT: return (float)v.i();
        case Type::LONG: return (float)v.l();
        case Type::FLOAT: return v.f();
        default: return (float)v.d();
    }
}
static int64_t as_long(const Val& v) {
    switch ((Type)v.t) {
        case Type::INT: return v.i();
        case Type::LONG: return v.l();
        case Type::FLOAT: { float x = v.f(); if (x != x) return 0; if (x >= 9.2233720368547758e18f) return INT64_MAX; if (x <= -9.2233720368547758e18f) return INT64_MIN; return (int64_t)x; }
        default: { double x = v.d(); if (x != x) return 0; if (x >= 9.2233720368547758e18) return INT64_MAX; if (x <= -9.2233720368547758e18) return INT64_MIN; return (int64_t)x; }
    }
}
static int32_t as_int(const Val& v) {
    switch ((Type)v.t) {
        case Type::INT: return v.i();
        case Type::LONG: return (int32_t)v.l();
        case Type::FLOAT: { float x = v.f(); if (x != x) return 0; if (x >= 2147483647.0f) return INT32_MAX; if (x <= -2147483648.0f) return INT32_MIN; return (int32_t)x; }
        default: { double x = v.d(); if (x != x) return 0; if (x >= 2147483647.0) return INT32_MAX; if (x <= -2147483648.0) return INT32_MIN; return (int32_t)x; }
    }
}

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

// Java Float.toString / Double.toString layout with shortest round-trip digits
static std::string java_real_to_string(double x, bool is_float) {
    if (x != x) return "NaN";
    if (std::isinf(x)) return x > 0 ? "Infinity" : "-Infinity";
    if (x == 0) return std::signbit(x) ? "-0.0" : "0.0";
    char buf[64];
    int prec = 1;
    for (; prec <= 17; ++prec) {
        std::snprintf(buf, sizeof buf, "%.*e", prec - 1, x);
        if (is_float ? (std::strtof(buf, nullptr) == (float)x) : (std::strtod(buf, nullptr) == x)) break;
    }
    // buf = d.ddddde[+-]XX
    std::string s(buf);
    bool neg = s[0] == '-';
    if (neg) s = s.substr(1);
    size_t epos = s.find('e');
    std::string mant = s.substr(0, epos);
    int exp10 = std::atoi(s.c_str() + epos + 1);
    std::string digits;
    for (char c : mant) if (c != '.') digits += c;
    while (digits.size() > 1 && digits.back() == '0') digits.pop_back();
    std::string out;
    double ax = std::fabs(x);
    if (ax >= 1e-3 && ax < 1e7) {
        int point = exp10 + 1;  // digits before the decimal point
        if (point <= 0) {
            out = "0." + std::string(-point, '0') + digits;
        } else if ((int)digits.size() <= point) {
            out = digits + std::string(point - digits.size(), '0') + ".0";
        } else {
            out = digits.substr(0, point) + "." + digits.substr(point);
        }
    } else {
        out = digits.substr(0, 1) + "." + (digits.size() > 1 ? digits.substr(1) : "0") + "E" + std::to_string(exp10);
    }
    return neg ? "-" + out : out;
}

// ------------------------------------------------------------------------------------------------
// intrusive ref counting (objects live while referenced, as under the JVM GC)
template <class T>
class Ref {
    T* p_ = nullptr;
   public:
    Ref() = default;
    Ref(std::nullptr_t) {}
    explicit Ref(T* p) : p_(p) { if (p_) ++p_->rc; }
    Ref(const Ref& o) : p_(o.p_) { if (p_) ++p_->rc; }
    Ref(Ref&& o) noexcept : p_(o.p_) { o.p_ = nullptr; }
    ~Ref() { release(); }
    Ref& operator=(const Ref& o) { if (o.p_) ++o.p_->rc; release(); p_ = o.p_; return *this; }
    Ref& operator=(Ref&& o) noexcept { if (this != &o) { release(); p_ = o.p_; o.p_ = nullptr; } return *this; }
    Ref& operator=(std::nullptr_t) { release(); return *this; }
    void release() { if (p_ && --p_->rc == 0) delete p_; p_ = nullptr; }
    T* get() const { return p_; }
    T* operator->() const { return p_; }
    explicit operator bool() const { return p_ != nullptr; }
    bool operator==(const Ref& o) const { return p_ == o.p_; }
    bool operator!=(const Ref& o) const { return p_ != o.p_; }
};

enum EvType : uint8_t { CURRENT = 0, EXPIRED = 1, TIMER = 2, RESET = 3 };

struct StreamEvent {
    int rc = 0;
    int64_t ts = 0;
    EvType type = CURRENT;
    std::vector<Val> data;
    Ref<StreamEvent> next;
    ~StreamEvent() {  // unlink iteratively to keep deep chains off the stack
        while (next && next->rc == 1) {
            Ref<StreamEvent> n = std::move(next->next);
            next = std::move(n);
        }
    }
};
using SEv = Ref<StreamEvent>;

struct StateEvent {
    int rc = 0;
    std::vector<SEv> se;        // streamEvents
    Ref<StateEvent> next;
    int64_t ts = -1;
    EvType type = CURRENT;
    std::vector<Val> out;       // outputData (multi-value outputs kept beside)
    std::vector<std::shared_ptr<std::vector<Val>>> out_list;
    int64_t id = 0;

    // StateEvent.getStreamEvent(int[] position) (StateEvent.java:138-182)
    StreamEvent* get(int chain, int idx) const {
        StreamEvent* e = se[chain].get();
        if (!e) return nullptr;
        if (idx >= 0) {
            for (int i = 1; i <= idx; ++i) {
                e = e->next.get();
                if (!e) return nullptr;
            }
        } else if (idx == sql::IDX_CURRENT) {
            while (e->next) e = e->next.get();
        } else if (idx == sql::IDX_LAST) {
            if (!e->next) return nullptr;
            while (e->next->next) e = e->next.get();
        } else {
            std::vector<StreamEvent*> lst;
            while (e) { lst.push_back(e); e = e->next.get(); }
            int k = (int)lst.size() + idx;
            if (k < 0) return nullptr;
            e = lst[k];
        }
        return e;
    }
    // addEvent / removeLastEvent (StateEvent.java:215-240)
    void addEvent(int pos, SEv ev) {
        StreamEvent* a = se[pos].get();
        if (!a) { se[pos] = ev; return; }
        while (a->next) a = a->next.get();
        a->next = ev;
    }
    void removeLastEvent(int pos) {
        StreamEvent* a = se[pos].get();
        if (a) {
            while (a->next) {
                if (!a->next->next) { a->next = nullptr; return; }
                a = a->next.get();
            }
            se[pos] = nullptr;
        }
    }
};
using StEv = Ref<StateEvent>;

// ComplexEventChunk<StateEvent> (event/ComplexEventChunk.java)
struct Chunk {
    StEv first, prevToLast, lastRet, last;
    static StEv lastEvent(const StEv& evs) {
        StateEvent* l = evs.get();
        while (l && l->next && l->next.get() != evs.get()) l = l->next.get();
        if (l && l->next.get() == evs.get()) l->next = nullptr;  // detach the loop
        return StEv(l);
    }
    void add(const StEv& evs) {
        if (!first) first = evs;
        else last->next = evs;
        last = lastEvent(evs);
    }
    bool hasNext() const {
        if (lastRet) return (bool)lastRet->next;
        if (prevToLast) return (bool)prevToLast->next;
        return (bool)first;
    }
    StEv next() {
        StEv r;
        if (lastRet) { r = lastRet->next; prevToLast = lastRet; }
        else if (prevToLast) r = prevToLast->next;
        else r = first;
        if (!r) throw OracleError("NoSuchElementException");
        lastRet = r;
        return r;
    }
    void remove() {
        if (!lastRet) throw OracleError("IllegalStateException");
        if (prevToLast) prevToLast->next = lastRet->next;
        else {
            first = lastRet->next;
            if (!first) last = nullptr;
        }
        lastRet->next = nullptr;
        lastRet = nullptr;
    }
    void clear() { prevToLast = nullptr; lastRet = nullptr; first = nullptr; last = nullptr; }
    void reset() { prevToLast = nullptr; lastRet = nullptr; }
};

// ------------------------------------------------------------------------------------------------
// JDK 8 java.util.HashMap<String, V> iteration-order emulation (list bins only)
static int32_t java_string_hash(const std::string& s) {
    uint32_t h = 0;
    size_t i = 0;
    while (i < s.size()) {  // UTF-8 -> UTF-16 code units
        uint32_t c = (unsigned char)s[i];
        uint32_t cp;
        if (c < 0x80) { cp = c; i += 1; }
        else if ((c >> 5) == 6 && i + 1 < s.size()) { cp = ((c & 0x1f) << 6) | (s[i + 1] & 0x3f); i += 2; }
        else if ((c >> 4) == 14 && i + 2 < s.size()) { cp = ((c & 0x0f) << 12) | ((s[i + 1] & 0x3f) << 6) | (s[i + 2] & 0x3f); i += 3; }
        else if (i + 3 < s.size()) { cp = ((c & 0x07) << 18) | ((s[i + 1] & 0x3f) << 12) | ((s[i + 2] & 0x3f) << 6) | (s[i + 3] & 0x3f); i += 4; }
        else { cp = c; i += 1; }
        if (cp >= 0x10000) {
            cp -= 0x10000;
            h = 31 * h + (0xD800 + (cp >> 10));
            h = 31 * h + (0xDC00 + (cp & 0x3ff));
        } else {
            h = 31 * h + cp;
        }
    }
    return (int32_t)h;
}

template <class V>
struct JHashMap {
    struct Node {
        int32_t hash;
        std::string key;
        V val;
        Node* next;
    };
    std::vector<Node*> table;
    size_t size = 0, threshold = 0;
    ~JHashMap() {
        for (Node* b : table)
            while (b) { Node* n = b->next; delete b; b = n; }
    }
    static int32_t spread(const std::string& k) {
        int32_t h = java_string_hash(k);
        return h ^ (int32_t)((uint32_t)h >> 16);
    }
    void resize() {
        size_t oldCap = table.size();
        if (oldCap == 0) {
            table.assign(16, nullptr);
            threshold = 12;
            return;
        }
        size_t newCap = oldCap * 2;
        std::vector<Node*> nt(newCap, nullptr);
        for (size_t j = 0; j < oldCap; ++j) {
            Node *loH = nullptr, *loT = nullptr, *hiH = nullptr, *hiT = nullptr;
            for (Node* e = table[j]; e;) {
                Node* nx = e->next;
                if ((e->hash & (int32_t)oldCap) == 0) { if (loT) loT->next = e; else loH = e; loT = e; }
                else { if (hiT) hiT->next = e; else hiH = e; hiT = e; }
                e = nx;
            }
            if (loT) { loT->next = nullptr; nt[j] = loH; }
            if (hiT) { hiT->next = nullptr; nt[j + oldCap] = hiH; }
        }
        table.swap(nt);
        threshold *= 2;
    }
    Node* find(const std::string& k) const {
        if (table.empty()) return nullptr;
        int32_t h = spread(k);
        for (Node* e = table[(table.size() - 1) & (uint32_t)h]; e; e = e->next)
            if (e->hash == h && e->key == k) return e;
        return nullptr;
    }
    // HashMap.computeIfAbsent (JDK 8): resize first when size > threshold; new node at the HEAD of its bin
    V& computeIfAbsent(const std::string& k, const std::function<V()>& make) {
        if (size > threshold || table.empty()) resize();
        int32_t h = spread(k);
        size_t i = (table.size() - 1) & (uint32_t)h;
        int binCount = 0;
        for (Node* e = table[i]; e; e = e->next) {
            if (e->hash == h && e->key == k) return e->val;
            ++binCount;
        }
        Node* n = new Node{h, k, make(), table[i]};
        table[i] = n;
        if (binCount >= 7 && table.size() < 64) resize();  // treeifyBin on a small table resizes
        ++size;
        return n->val;
    }
    void remove(const std::string& k) {
        if (table.empty()) return;
        int32_t h = spread(k);
        size_t i = (table.size() - 1) & (uint32_t)h;
        Node* prev = nullptr;
        for (Node* e = table[i]; e; prev = e, e = e->next) {
            if (e->hash == h && e->key == k) {
                if (prev) prev->next = e->next;
                else table[i] = e->next;
                delete e;
                --size;
                return;
            }
        }
    }
    template <class F>
    void for_each(F f) {
        for (size_t b = 0; b < table.size(); ++b)
            for (Node* e = table[b]; e; e = e->next) f(e->key, e->val);
    }
};

// PartitionState.partitionKeys (PartitionRuntimeImpl.java:423) is a java.util.concurrent.ConcurrentHashMap
// <String, Long>; PartitionStreamReceiver.send(ComplexEvent) (:274-283) walks getPartitionKeys() = new
// HashSet<>(partitionKeys.keySet()) (PartitionRuntimeImpl.java:404-407). Both iteration orders, JDK 8, single-threaded:
//   ConcurrentHashMap: table of 16 on the first put (initTable); putVal appends a new key at the TAIL of its bin;
//     after a put that makes count >= sizeCtl (0.75 n) the table doubles (addCount -> transfer); a put that walked
//     >= 8 nodes of a bin calls treeifyBin, which on a table < 64 presizes instead (tryPresize(n << 1): doubles
//     until tableSizeFor(3n + 1) <= sizeCtl). transfer splits a list bin by its `lastRun`: the maximal tail whose
//     nodes all go to one side keeps its order and heads that side; every node before it is PREPENDED to its side
//     (so their order reverses). Iteration: bins 0..n-1, each bin's list in order. Tree bins (>= 8 keys in one bin
//     of a table >= 64) are not modelled: such a bin throws.
//   HashSet(Collection c): new HashMap(max((int)(c.size() / .75f) + 1, 16)) (capacity tableSizeFor of that), then
//     add() of every key in the CHM's iteration order; HashMap.putVal appends at the tail of its bin (no resize
//     happens below 0.75 load; a bin reaching 9 keys would treeify and is not modelled: throws).
struct JavaCHM {
    struct Node {
        int32_t hash;  // spread(h) = (h ^ h >>> 16) & 0x7fffffff
        std::string key;
    };
    std::vector<std::vector<Node>> table;
    int64_t count = 0, sizeCtl = 0;
    bool tree = false;  // some bin treeified (ConcurrentHashMap.treeifyBin on a table >= 64)
    static int32_t spread(const std::string& k) {
        int32_t h = java_string_hash(k);
        return (h ^ (int32_t)((uint32_t)h >> 16)) & 0x7fffffff;
    }
    static int64_t tableSizeFor(int64_t c) {
        int64_t n = 1;
        while (n < c) n <<= 1;
        return n;
    }
    void transfer() {  // ConcurrentHashMap.transfer, one thread
        const size_t n = table.size();
        std::vector<std::vector<Node>> nt(2 * n);
        for (size_t i = 0; i < n; ++i) {
            std::vector<Node>& f = table[i];
            if (f.empty()) continue;
            size_t lastRun = 0;
            bool runBit = (f[0].hash & (int32_t)n) != 0;
            for (size_t p = 1; p < f.size(); ++p) {
                const bool b = (f[p].hash & (int32_t)n) != 0;
                if (b != runBit) { runBit = b; lastRun = p; }
            }
            std::vector<Node> ln, hn;  // built front to back: the lastRun tail, then the prefix prepended
            std::vector<Node>& run = runBit ? hn : ln;
            run.assign(f.begin() + lastRun, f.end());
            for (size_t p = 0; p < lastRun; ++p) {
                std::vector<Node>& side = (f[p].hash & (int32_t)n) ? hn : ln;
                side.insert(side.begin(), f[p]);
            }
            nt[i] = std::move(ln);
            nt[i + n] = std::move(hn);
        }
        table.swap(nt);
        sizeCtl = (int64_t)(2 * n) - (int64_t)(n >> 1);  // 0.75 * 2n
    }
    void put(const std::string& k) {  // putVal(k, v, false) then addCount
        if (table.empty()) {
            table.assign(16, {});
            sizeCtl = 12;
        }
        const int32_t h = spread(k);
        std::vector<Node>& bin = table[(table.size() - 1) & (uint32_t)h];
        int binCount = 0;
        bool found = false;
        if (!bin.empty()) {
            binCount = 1;
            for (size_t p = 0;; ++binCount, ++p) {
                if (bin[p].hash == h && bin[p].key == k) { found = true; break; }
                if (p + 1 == bin.size()) { bin.push_back(Node{h, k}); break; }
            }
        } else {
            bin.push_back(Node{h, k});
        }
        if (binCount >= 8) {  // treeifyBin
            if (table.size() < 64) {  // tryPresize(n << 1)
                const int64_t c = tableSizeFor(3 * (int64_t)table.size() + 1);
                while (!(c <= sizeCtl)) transfer();
            } else {
                tree = true;  // a TreeBin: only its iteration order is not modelled (hashset_order refuses then)
            }
        }
        if (found) return;
        if (++count >= sizeCtl) transfer();
    }
    void remove(const std::string& k) {  // replaceNode(k, null, null): unlinked, the table never shrinks
        if (table.empty()) return;
        const int32_t h = spread(k);
        std::vector<Node>& bin = table[(table.size() - 1) & (uint32_t)h];
        for (size_t p = 0; p < bin.size(); ++p)
            if (bin[p].hash == h && bin[p].key == k) {
                bin.erase(bin.begin() + p);
                --count;
                return;
            }
    }
    // new HashSet<>(keySet()) iterated
    std::vector<std::string> hashset_order() const {
        if (tree) throw OracleError("partition key order: a ConcurrentHashMap tree bin (not modelled)");
        int64_t cap = tableSizeFor(std::max<int64_t>((int64_t)((float)count / 0.75f) + 1, 16));
        std::vector<std::vector<const Node*>> hs((size_t)cap);
        for (const auto& bin : table)
            for (const Node& nd : bin) {
                auto& b = hs[(size_t)(nd.hash & (int32_t)(cap - 1))];
                b.push_back(&nd);
                if (b.size() >= 9) {  // putVal's treeifyBin: a table < 64 resizes (order-preserving split)
                    if (cap >= 64) throw OracleError("partition key order: a HashMap tree bin (not modelled)");
                    std::vector<std::vector<const Node*>> nt((size_t)cap * 2);
                    for (const auto& ob : hs)
                        for (const Node* x : ob) nt[(size_t)(x->hash & (int32_t)(2 * cap - 1))].push_back(x);
                    hs.swap(nt);
                    cap *= 2;
                }
            }
        std::vector<std::string> out;
        out.reserve((size_t)count);
        for (const auto& b : hs)
            for (const Node* x : b) out.push_back(x->key);
        return out;
    }
};

// ------------------------------------------------------------------------------------------------
struct Engine;
struct Ctx {
    bool has_key = false;
    std::string key;  // SiddhiAppContext partition flow id (ThreadLocal)
};

// StreamPreStateProcessor.StreamPreState (+ Count and Logical/Absent subclass fields)
struct PreState {
    Chunk cur;
    std::list<StEv> pending, newAndEvery;
    bool stateChanged = false, initialized = false, started = false;
    bool successCondition = false, startStateReset = false;  // CountStreamPreState
    int64_t lastScheduledTime = 0;                           // AbsentStreamPreState
    int64_t lastArrivalTime = 0;                             // AbsentLogicalPreStateProcessor.LogicalStreamPreState
    bool active = true;
    int activeUseCount = 0;
    // StreamPreState.canDestroy :444-448 (&& lastArrivalTime == 0: LogicalStreamPreState.canDestroy :403-405;
    // the field stays 0 for every other kind)
    bool canDestroy() const {
        return !cur.first && pending.empty() && newAndEvery.empty() && !initialized && lastArrivalTime == 0;
    }
};
using PS = std::shared_ptr<PreState>;

// PartitionSyncStateHolder / SingleSyncStateHolder for processor states
struct PreStateHolder {
    Ctx* ctx;
    bool partitioned;
    PS single;
    std::unordered_map<std::string, PS> map;
    PS get() {
        if (!partitioned) {
            if (!single) single = std::make_shared<PreState>();
            return single;
        }
        PS& p = map[ctx->key];
        if (!p) p = std::make_shared<PreState>();
        p->activeUseCount++;
        return p;
    }
    void ret(const PS& s) {
        if (!partitioned) return;
        s->activeUseCount--;
        if (s->activeUseCount == 0) {
            if (s->canDestroy()) {
                auto it = map.find(ctx->key);
                if (it != map.end() && it->second == s) map.erase(it);
            }
        } else if (s->activeUseCount < 0) {
            throw OracleError("State active count has reached less then zero");
        }
    }
};
struct Hold {  // scoped getState()/returnState()
    PreStateHolder& h;
    PS s;
    explicit Hold(PreStateHolder& hh) : h(hh), s(hh.get()) {}
    ~Hold() { h.ret(s); }
    PreState* operator->() { return s.get(); }
};

// ------------------------------------------------------------------------------------------------
// executors
struct Exec {
    Type rt = Type::BOOL;
    virtual ~Exec() {}
    virtual Val exec(StateEvent* e) = 0;
};
using ExecP = std::unique_ptr<Exec>;

struct ConstExec : Exec {
    Val v;
    Val exec(StateEvent*) override { return v; }
};
// VariableExpressionExecutor over a StateEvent position [chain, index-in-chain, attribute]
struct VarExec : Exec {
    int chain, idx, attr;
    Val exec(StateEvent* e) override {
        StreamEvent* s = e->get(chain, idx);
        if (!s) return vnull(rt);
        return s->data[attr];
    }
};
// MultiValueVariableFunctionExecutor: list of the attribute over the whole chain (selector only)
struct MultiVarExec : Exec {
    int chain, attr;
    Val exec(StateEvent*) override { return vnull(rt); }
    std::shared_ptr<std::vector<Val>> list(StateEvent* e) {
        auto l = std::make_shared<std::vector<Val>>();
        for (StreamEvent* s = e->se[chain].get(); s; s = s->next.get()) l->push_back(s->data[attr]);
        return l;
    }
};
// a having-scope variable that names an output attribute (ExpressionParser.parseVariable HAVING_STATE branch)
struct OutVarExec : Exec {
    int j;
    Val exec(StateEvent* e) override { return e->out[j]; }
};
struct AndExec : Exec {  // AndConditionExpressionExecutor.java:65-74
    ExecP l, r;
    Val exec(StateEvent* e) override {
        Val a = l->exec(e);
        if (!a.null && a.b()) {
            Val b = r->exec(e);
            if (!b.null && b.b()) return vB(true);
        }
        return vB(false);
    }
};
struct OrExec : Exec {  // OrConditionExpressionExecutor.java:65-76
    ExecP l, r;
    Val exec(StateEvent* e) override {
        Val a = l->exec(e);
        if (!a.null && a.b()) return vB(true);
        Val b = r->exec(e);
        if (!b.null && b.b()) return vB(true);
        return vB(false);
    }
};
struct NotExec : Exec {  // NotConditionExpressionExecutor.java:43-50 (null -> TRUE)
    ExecP x;
    Val exec(StateEvent* e) override {
        Val a = x->exec(e);
        return vB(!(!a.null && a.b()));
    }
};
struct BoolExec : Exec {  // BoolConditionExpressionExecutor (bool attribute used as a condition)
    ExecP x;
    Val exec(StateEvent* e) override {
        Val a = x->exec(e);
        if (a.null) return vB(false);
        return vB(a.b());
    }
};
struct IsNullExec : Exec {
    ExecP x;
    Val exec(StateEvent* e) override { return vB(x->exec(e).null); }
};
struct IsNullStreamExec : Exec {
    int chain, idx;
    Val exec(StateEvent* e) override { return vB(e->get(chain, idx) == nullptr); }
};
// compare executors (executor/condition/compare/**): per-(left,right)-type Java semantics
struct CmpExec : Exec {
    sql::CmpOp op;
    Type lt, rtp;
    ExecP l, r;
    template <class T>
    static bool cmp(sql::CmpOp op, T a, T b) {
        switch (op) {
            case sql::CmpOp::EQ: return a == b;
            case sql::CmpOp::NE: return a != b;
            case sql::CmpOp::GT: return a > b;
            case sql::CmpOp::GE: return a >= b;
            case sql::CmpOp::LT: return a < b;
            default: return a <= b;
        }
    }
    Val exec(StateEvent* e) override {
        Val a = l->exec(e), b = r->exec(e);
        if (a.null || b.null) return vB(false);  // CompareConditionExpressionExecutor.java:38-42
        if (lt == Type::STRING) return vB(op == sql::CmpOp::EQ ? a.raw == b.raw : a.raw != b.raw);
        if (lt == Type::BOOL) return vB(op == sql::CmpOp::EQ ? a.b() == b.b() : a.b() != b.b());
        bool eqop = op == sql::CmpOp::EQ || op == sql::CmpOp::NE;
        auto isT = [](Type t, Type x) { return t == x; };
        if (isT(lt, Type::DOUBLE) || isT(rtp, Type::DOUBLE)) return vB(cmp(op, as_double(a), as_double(b)));
        if (isT(lt, Type::FLOAT) || isT(rtp, Type::FLOAT)) {
            // Equal/NotEqual Float-Long and Long-Float compare in double (EqualCompare...FloatLong.java)
            if (eqop && (lt == Type::LONG || rtp == Type::LONG)) return vB(cmp(op, as_double(a), as_double(b)));
            return vB(cmp(op, as_float(a), as_float(b)));
        }
        if (isT(lt, Type::LONG) || isT(rtp, Type::LONG)) return vB(cmp(op, as_long(a), as_long(b)));
        return vB(cmp(op, a.i(), b.i()));
    }
};
// math executors (executor/math/**): result type by promotion (ExpressionParser.java:1488-1520)
struct MathExec : Exec {
    sql::ExprKind k;
    ExecP l, r;
    Val exec(StateEvent* e) override {
        Val a = l->exec(e), b = r->exec(e);
        if (a.null || b.null) return vnull(rt);
        switch (rt) {
            case Type::DOUBLE: {
                double x = as_double(a), y = as_double(b);
                switch (k) {
                    case sql::ExprKind::ADD: return vD(x + y);
                    case sql::ExprKind::SUB: return vD(x - y);
                    case sql::ExprKind::MUL: return vD(x * y);
                    case sql::ExprKind::DIV: if (y == 0.0) return vnull(rt); return vD(x / y);
                    default: if (y == 0.0) return vnull(rt); return vD(std::fmod(x, y));
                }
            }
            case Type::FLOAT: {
                float x = as_float(a), y = as_float(b);
                switch (k) {
                    case sql::ExprKind::ADD: return vF(x + y);
                    case sql::ExprKind::SUB: return vF(x - y);
                    case sql::ExprKind::MUL: return vF(x * y);
                    case sql::ExprKind::DIV: if (y == 0.0f) return vnull(rt); return vF(x / y);
                    default: if (y == 0.0f) return vnull(rt); return vF(std::fmod(x, y));
                }
            }
            case Type::LONG: {
                int64_t x = as_long(a), y = as_long(b);
                uint64_t ux = (uint64_t)x, uy = (uint64_t)y;
                switch (k) {
                    case sql::ExprKind::ADD: return vL((int64_t)(ux + uy));
                    case sql::ExprKind::SUB: return vL((int64_t)(ux - uy));
                    case sql::ExprKind::MUL: return vL((int64_t)(ux * uy));
                    case sql::ExprKind::DIV: if (y == 0) return vnull(rt); if (x == INT64_MIN && y == -1) return vL(x); return vL(x / y);
                    default: if (y == 0) return vnull(rt); if (y == -1) return vL(0); return vL(x % y);
                }
            }
            default: {
                int32_t x = as_int(a), y = as_int(b);
                uint32_t ux = (uint32_t)x, uy = (uint32_t)y;
                switch (k) {
                    case sql::ExprKind::ADD: return vI((int32_t)(ux + uy));
                    case sql::ExprKind::SUB: return vI((int32_t)(ux - uy));
                    case sql::ExprKind::MUL: return vI((int32_t)(ux * uy));
                    case sql::ExprKind::DIV: if (y == 0) return vnull(rt); if (x == INT32_MIN && y == -1) return vI(x); return vI(x / y);
                    default: if (y == 0) return vnull(rt); if (y == -1) return vI(0); return vI(x % y);
                }
            }
        }
    }
};

// function executors (core/executor/function/*.java). FunctionExecutor.execute evaluates every argument first.
struct IfThenElseExec : Exec {  // IfThenElseFunctionExecutor.execute: Boolean.TRUE.equals(data[0]) ? data[1] : data[2]
    ExecP c, a, b;
    Val exec(StateEvent* e) override {
        Val cv = c->exec(e), av = a->exec(e), bv = b->exec(e);
        return (!cv.null && cv.b()) ? av : bv;
    }
};
struct CoalesceExec : Exec {  // CoalesceFunctionExecutor / DefaultFunctionExecutor: the first non-null argument
    std::vector<ExecP> xs;
    Val exec(StateEvent* e) override {
        std::vector<Val> v;
        for (auto& x : xs) v.push_back(x->exec(e));
        for (auto& x : v)
            if (!x.null) return x;
        return vnull(rt);
    }
};
struct InstanceOfExec : Exec {  // InstanceOf{Boolean,Double,Float,Integer,Long,String}FunctionExecutor: data instanceof T
    ExecP x;
    Type target;
    Val exec(StateEvent* e) override {
        Val v = x->exec(e);
        return vB(!v.null && (Type)v.t == target);
    }
};
static int32_t java_d2i(double d) {  // JLS 5.1.3 narrowing: NaN -> 0, saturating
    if (d != d) return 0;
    if (d >= 2147483647.0) return INT32_MAX;
    if (d <= -2147483648.0) return INT32_MIN;
    return (int32_t)d;
}
static int64_t java_d2l(double d) {
    if (d != d) return 0;
    if (d >= 9223372036854775807.0) return INT64_MAX;
    if (d <= -9223372036854775808.0) return INT64_MIN;
    return (int64_t)d;
}
// MaximumFunctionExecutor / MinimumFunctionExecutor.execute(Object[]): a double running max starting at
// Double.MIN_VALUE (the smallest POSITIVE double) / min starting at Double.MAX_VALUE; a null argument counts as
// that start value; the result is cast back to the argument type. One argument: execute(Object) returns it as is.
struct MaxMinExec : Exec {
    bool is_max = true;
    std::vector<ExecP> xs;
    Val exec(StateEvent* e) override {
        std::vector<Val> v;
        for (auto& x : xs) v.push_back(x->exec(e));
        if (v.size() == 1) return v[0];
        const double start = is_max ? 4.9e-324 : 1.7976931348623157e308;
        double best = start;
        for (auto& x : v) {
            const double value = x.null ? start : as_double(x);
            if (is_max ? value > best : value < best) best = value;
        }
        switch (rt) {
            case Type::INT: return vI(java_d2i(best));
            case Type::LONG: return vL(java_d2l(best));
            case Type::FLOAT: return vF((float)best);
            default: return vD(best);
        }
    }
};

// attribute aggregators (core/query/selector/attribute/aggregator/*AttributeAggregatorExecutor.java) with their
// state per partition key (the selector's state holder is partition-aware). Pattern outputs reach the selector
// as CURRENT events only, so the states only ever add (EXPIRED: processRemove, restated for count/sum/avg).
struct AggExec : Exec {
    enum K { COUNT, SUM, AVG, MIN, MAX } k = COUNT;
    ExecP arg;  // null for count()
    Type at = Type::LONG;
    const Ctx* ctx = nullptr;
    bool partitioned = false;
    struct St {
        int64_t count = 0;
        int64_t lsum = 0;
        double dsum = 0;
        bool has = false;  // MIN/MAX: minValue != null
        Val m;
    };
    std::unordered_map<std::string, St> states;
    Val exec(StateEvent* e) override {
        St& s = states[partitioned ? ctx->key : std::string()];
        const bool add = e->type != EXPIRED;
        if (k == COUNT) {  // CountAttributeAggregatorExecutor.processAdd / processRemove
            s.count += add ? 1 : -1;
            return vL(s.count);
        }
        Val v = arg->exec(e);
        const bool integral = at == Type::INT || at == Type::LONG;
        if (k == SUM) {  // SumAttributeAggregatorExecutor: AggregatorState{Int->Long, Long, Float->Double, Double}
            if (!v.null) {
                if (integral) s.lsum = (int64_t)((uint64_t)s.lsum + (uint64_t)(add ? as_long(v) : -as_long(v)));
                else s.dsum = add ? s.dsum + as_double(v) : s.dsum - as_double(v);
                s.count += add ? 1 : -1;
            }
            if (s.count == 0) return vnull(rt);  // currentValue / processRemove at count 0
            return integral ? vL(s.lsum) : vD(s.dsum);
        }
        if (k == AVG) {  // AvgAttributeAggregatorExecutor: double value, long count
            if (!v.null) {
                s.count += add ? 1 : -1;
                s.dsum = add ? s.dsum + as_double(v) : s.dsum - as_double(v);
            }
            if (s.count == 0) return vnull(rt);
            return vD(s.dsum / (double)s.count);
        }
        // Min/MaxAttributeAggregatorExecutor (and the *Forever variants): minValue == null || minValue > value
        if (!add) throw OracleError("unsupported: min/max of expired events on the pattern path");
        if (!v.null) {
            bool take = !s.has;
            if (s.has) {
                switch (at) {
                    case Type::INT: take = k == MIN ? s.m.i() > v.i() : s.m.i() < v.i(); break;
                    case Type::LONG: take = k == MIN ? s.m.l() > v.l() : s.m.l() < v.l(); break;
                    case Type::FLOAT: take = k == MIN ? s.m.f() > v.f() : s.m.f() < v.f(); break;
                    default: take = k == MIN ? s.m.d() > v.d() : s.m.d() < v.d(); break;
                }
            }
            if (take) {
                s.m = v;
                s.has = true;
            }
        }
        return s.has ? s.m : vnull(rt);
    }
};

// ------------------------------------------------------------------------------------------------
// processors
struct Processor {
    Processor* nextProcessor = nullptr;
    virtual ~Processor() {}
    virtual void process(Chunk& c) = 0;
    virtual void setNextProcessor(Processor* p) { nextProcessor = p; }
    void setToLast(Processor* p) {
        if (!nextProcessor) setNextProcessor(p);
        else nextProcessor->setToLast(p);
    }
};

// FilterProcessor.java:48-60
struct FilterProc : Processor {
    ExecP cond;
    void process(Chunk& c) override {
        c.reset();
        while (c.hasNext()) {
            StEv ev = c.next();
            Val r = cond->exec(ev.get());
            if (r.null || !r.b()) c.remove();
        }
        if (c.first) nextProcessor->process(c);
    }
};

struct PreProc;
struct CountPre;
struct Selector;

// StreamPostStateProcessor.java
struct Post : Processor {
    PreProc* nextStatePre = nullptr;
    PreProc* nextEveryStatePre = nullptr;
    PreProc* thisPre = nullptr;
    int stateId = 0;
    CountPre* callbackPre = nullptr;
    bool isEventReturned = false;
    void process(Chunk& c) override {
        c.reset();
        if (c.hasNext()) {
            StEv se = c.next();
            processSE(se, c);
        }
        c.clear();
    }
    virtual void processSE(StEv se, Chunk& c);
    virtual void setNextStatePreProcessor(PreProc* p) { nextStatePre = p; }
    virtual void setNextEveryStatePreProcessor(PreProc* p) { nextEveryStatePre = p; }
    void setCallbackPreStateProcessor(CountPre* c) { callbackPre = c; }
};

enum class PreKind : uint8_t { STREAM, COUNT, LOGICAL, ABSENT };

struct Scheduler;

// StreamPreStateProcessor.java
struct PreProc : Processor {
    Engine* eng = nullptr;
    PreKind kind = PreKind::STREAM;
    int stateId = 0;
    bool isStartState = false;
    sql::StateType stateType = sql::StateType::PATTERN;
    int64_t withinTime = -1;  // SiddhiConstants.UNKNOWN_STATE
    std::vector<int> startStateIds;
    PreProc* withinEveryPre = nullptr;
    Post* thisPost = nullptr;
    Post* thisLast = nullptr;
    PreStateHolder holder;
    int nstates = 0;  // MetaStateEvent stream event count
    int noutputs = 0;
    int nattrs = 0;   // attributes of this state's stream (StreamEventFactory.newInstance output size)

    void process(Chunk&) override { throw OracleError("process method of StreamPreStateProcessor should not be called"); }
    virtual bool isAbsent() const { return false; }

    bool isExpired(StateEvent* se, int64_t ts) const {
        if (withinTime != -1) {
            for (int id : startStateIds) {
                StreamEvent* s = se->se[id].get();
                if (s && std::llabs(s->ts - ts) > withinTime) return true;
            }
        }
        return false;
    }
    StEv newStateEvent() const {
        StEv se(new StateEvent());
        se->se.resize(nstates);
        se->out.resize(noutputs);
        se->out_list.resize(noutputs);
        return se;
    }
    StEv cloneStateEvent(const StEv& o) const {  // StateEventCloner.copyStateEvent
        StEv n = newStateEvent();
        n->out = o->out;
        n->out_list = o->out_list;
        for (int i = 0; i < nstates; ++i) n->se[i] = o->se[i];
        n->type = o->type;
        n->ts = o->ts;
        n->id = o->id;
        return n;
    }
    static SEv copyStreamEvent(const SEv& e) {  // StreamEventCloner.copyStreamEvent
        SEv n(new StreamEvent());
        n->data = e->data;
        n->type = e->type;
        n->ts = e->ts;
        return n;
    }
    void processSE(const StEv& se) {  // process(StateEvent) :131-142
        Hold st(holder);
        st->cur.add(se);
        st->cur.reset();
        st->stateChanged = false;
        nextProcessor->process(st->cur);
        st->cur.reset();
    }
    virtual void init() {  // :178-194
        Hold st(holder);
        if (isStartState && (!st->initialized || thisPost->nextEveryStatePre != nullptr ||
                             (stateType == sql::StateType::SEQUENCE && thisPost->nextStatePre &&
                              thisPost->nextStatePre->isAbsent()))) {
            StEv se = newStateEvent();
            addState(se);
            st->initialized = true;
        }
    }
    void addState(const StEv& se) {
        Hold st(holder);
        addStateImpl(se, st.s);
    }
    virtual void addStateImpl(const StEv& se, const PS& st) {  // :214-227
        if (stateType == sql::StateType::SEQUENCE) {
            if (st->newAndEvery.empty()) st->newAndEvery.push_back(se);
        } else {
            st->newAndEvery.push_back(se);
        }
    }
    virtual void addEveryState(const StEv& se) {  // :230-247
        StEv cl = cloneStateEvent(se);
        cl->type = CURRENT;
        for (int i = stateId; i < (int)cl->se.size(); ++i) cl->se[i] = nullptr;
        Hold st(holder);
        st->newAndEvery.push_back(cl);
    }
    void stateChanged() {
        Hold st(holder);
        st->stateChanged = true;
    }
    bool pendingEmpty() {
        Hold st(holder);
        return st->pending.empty();
    }
    size_t pendingSize() {
        Hold st(holder);
        return st->pending.size();
    }
    void clearPending() {
        Hold st(holder);
        st->pending.clear();
    }
    virtual void resetState() {  // :288-305
        Hold st(holder);
        st->pending.clear();
        if (isStartState && st->newAndEvery.empty()) {
            if (stateType == sql::StateType::SEQUENCE && thisPost->nextEveryStatePre == nullptr) {
                if (!thisPost->nextStatePre) throw OracleError("NullPointerException in resetState");
                if (!thisPost->nextStatePre->pendingEmpty()) return;
            }
            init();
        }
    }
    static void sortByTime(std::list<StEv>& l) {  // eventTimeComparator, stable (List.sort / TimSort)
        std::vector<StEv> v(l.begin(), l.end());
        std::stable_sort(v.begin(), v.end(), [](const StEv& a, const StEv& b) {
            int64_t x = a->ts, y = b->ts;
            if (x == -1) return false;
            if (y == -1) return true;
            return x < y;
        });
        l.assign(v.begin(), v.end());
    }
    virtual void updateState() {  // :308-323
        Hold st(holder);
        sortByTime(st->newAndEvery);
        st->pending.splice(st->pending.end(), st->newAndEvery);
    }
    virtual void expireEvents(int64_t ts) {  // :326-361
        Hold st(holder);
        StEv expired;
        for (auto it = st->pending.begin(); it != st->pending.end();) {
            StEv se = *it;
            if (isExpired(se.get(), ts)) {
                it = st->pending.erase(it);
                if (se->type != EXPIRED) { se->type = EXPIRED; expired = se; }
            } else {
                break;
            }
        }
        for (auto it = st->newAndEvery.begin(); it != st->newAndEvery.end();) {
            StEv se = *it;
            if (isExpired(se.get(), ts)) {
                it = st->newAndEvery.erase(it);
                if (se->type != EXPIRED) { se->type = EXPIRED; expired = se; }
            } else {
                ++it;
            }
        }
        if (expired && withinEveryPre) {
            withinEveryPre->addEveryState(expired);
            withinEveryPre->updateState();
        }
    }
    virtual bool removeOnNoStateChange() const { return stateType == sql::StateType::SEQUENCE; }
    virtual Chunk processAndReturn(const SEv& ev);  // :364-403
    virtual void partitionCreated() {}
    // EntryValveProcessor -> process(ComplexEventChunk) of a TIMER event (absent processors only)
    virtual void processTimer(int64_t) { throw OracleError("timer delivered to a non-absent processor"); }
    virtual void updateLastArrivalTime(int64_t) { throw OracleError("updateLastArrivalTime on a non-absent processor"); }
    SEv emptyStreamEvent() const {  // StreamEventFactory.newInstance(): timestamp -1, all attributes null
        SEv n(new StreamEvent());
        n->ts = -1;
        n->data.resize(nattrs);
        return n;
    }
};

// CountPreStateProcessor.java
struct CountPost;
struct CountPre : PreProc {
    int minCount = 0, maxCount = 0;
    CountPost* countPost = nullptr;
    int resetDepth = 0;
    Chunk processAndReturn(const SEv& ev) override;
    void successCondition() {
        Hold st(holder);
        st->successCondition = true;
    }
    void addStateImpl(const StEv& se, const PS& st) override;
    void startStateReset();
    void updateState() override {
        Hold st(holder);
        if (st->startStateReset) {
            st->startStateReset = false;
            init();
        }
        PreProc::updateState();
    }
};

// StreamPostStateProcessor.process(StateEvent, chunk) :64-83
void Post::processSE(StEv se, Chunk& c) {
    thisPre->stateChanged();
    StreamEvent* s = se->se[stateId].get();
    se->ts = s->ts;
    if (nextProcessor) {
        c.reset();
        isEventReturned = true;
    }
    if (nextStatePre) nextStatePre->addState(se);
    if (nextEveryStatePre) nextEveryStatePre->addEveryState(se);
    if (callbackPre) callbackPre->startStateReset();
}

// CountPostStateProcessor.java
struct CountPost : Post {
    int minCount = 0, maxCount = 0;
    void processSE(StEv se, Chunk& c) override {
        StreamEvent* s = se->se[stateId].get();
        int n = 1;
        while (s->next) { ++n; s = s->next.get(); }
        static_cast<CountPre*>(thisPre)->successCondition();
        se->ts = s->ts;
        if (n >= minCount) {
            if (thisPre->stateType == sql::StateType::SEQUENCE) {
                if (nextStatePre) nextStatePre->addState(se);
                if (n != maxCount) thisPre->addState(se);
            } else if (n == minCount) {
                processMinCountReached(se, c);
            }
            if (n == maxCount) thisPre->stateChanged();
        }
    }
    void processMinCountReached(const StEv& se, Chunk& c) {
        if (nextProcessor) {
            thisPre->stateChanged();
            c.reset();
            isEventReturned = true;
        }
        if (nextStatePre) nextStatePre->addState(se);
        if (nextEveryStatePre) nextEveryStatePre->addEveryState(se);
    }
    void setNextStatePreProcessor(PreProc* p) override {
        nextStatePre = p;
        if (thisPre->isStartState && thisPre->stateType == sql::StateType::SEQUENCE && minCount == 0)
            p->thisPost->setCallbackPreStateProcessor(static_cast<CountPre*>(thisPre));
    }
};

void CountPre::addStateImpl(const StEv& se, const PS& st) {  // CountPreStateProcessor.java:97-125
    if (stateType == sql::StateType::SEQUENCE) {
        if (st->newAndEvery.empty()) st->newAndEvery.push_back(se);
    } else {
        st->newAndEvery.push_back(se);
    }
    if (minCount == 0 && !se->se[stateId]) {
        Chunk& ch = st->cur;
        ch.clear();
        ch.add(se);
        countPost->processMinCountReached(se, ch);
        ch.clear();
    }
}

void CountPre::startStateReset() {  // :168-181
    Hold st(holder);
    st->startStateReset = true;
    if (thisPost->callbackPre) {
        if (++resetDepth > 64) throw OracleError("StackOverflowError in CountPreStateProcessor.startStateReset");
        static_cast<CountPre*>(countPost->thisPre)->startStateReset();
        --resetDepth;
    }
}

// StreamPreStateProcessor.processAndReturn :364-403
Chunk PreProc::processAndReturn(const SEv& ev) {
    Chunk ret;
    Hold st(holder);
    auto& lst = st->pending;
    for (auto it = lst.begin(); it != lst.end();) {
        StEv se = *it;
        se->se[stateId] = copyStreamEvent(ev);
        processSE(se);
        if (thisLast->isEventReturned) {
            thisLast->isEventReturned = false;
            ret.add(se);
        }
        if (st->stateChanged) {
            it = lst.erase(it);
        } else {
            if (stateType == sql::StateType::PATTERN) {
                se->se[stateId] = nullptr;
                ++it;
            } else {
                se->se[stateId] = nullptr;
                if (removeOnNoStateChange()) it = lst.erase(it);
                else ++it;
                if (thisPost->callbackPre) thisPost->callbackPre->startStateReset();
            }
        }
    }
    return ret;
}

// CountPreStateProcessor.processAndReturn :53-95
Chunk CountPre::processAndReturn(const SEv& ev) {
    Chunk ret;
    Hold st(holder);
    auto& lst = st->pending;
    for (auto it = lst.begin(); it != lst.end();) {
        StEv se = *it;
        auto nextProcessed = [&](int pos) { return (int)se->se.size() > pos && se->se[pos]; };
        if (nextProcessed(stateId + 1)) { it = lst.erase(it); continue; }
        if (nextProcessed(stateId + 2)) { it = lst.erase(it); continue; }
        se->addEvent(stateId, copyStreamEvent(ev));
        st->successCondition = false;
        processSE(se);
        if (thisLast->isEventReturned) {
            thisLast->isEventReturned = false;
            ret.add(se);
        }
        bool erased = false;
        if (st->stateChanged) { it = lst.erase(it); erased = true; }
        if (!st->successCondition) {
            if (stateType == sql::StateType::PATTERN) {
                se->removeLastEvent(stateId);
            } else {
                se->removeLastEvent(stateId);
                if (erased) throw OracleError("IllegalStateException (iterator.remove twice)");
                it = lst.erase(it);
                erased = true;
            }
        }
        if (!erased) ++it;
    }
    return ret;
}

// LogicalPreStateProcessor.java / LogicalPostStateProcessor.java
struct LogicalPre : PreProc {
    sql::LogicalType logicalType = sql::LogicalType::AND;
    LogicalPre* partner = nullptr;
    bool newAndEveryEmpty() {
        Hold st(holder);
        return st->newAndEvery.empty();
    }
    void removeFromPending(const StEv& se) {  // getPendingStateEventList().remove(stateEvent): first occurrence
        Hold st(holder);
        for (auto it = st->pending.begin(); it != st->pending.end(); ++it)
            if (*it == se) { st->pending.erase(it); return; }
    }
    void addToNewAndEvery(const StEv& se) {
        Hold st(holder);
        st->newAndEvery.push_back(se);
    }
    void moveAllNewAndEveryToPending() {
        Hold st(holder);
        sortByTime(st->newAndEvery);
        st->pending.splice(st->pending.end(), st->newAndEvery);
    }
    void addStateImpl(const StEv& se, const PS& st) override {  // :43-62
        if (isStartState || stateType == sql::StateType::SEQUENCE) {
            if (st->newAndEvery.empty()) st->newAndEvery.push_back(se);
            if (partner && partner->newAndEveryEmpty()) partner->addToNewAndEvery(se);
        } else {
            st->newAndEvery.push_back(se);
            if (partner) partner->addToNewAndEvery(se);
        }
    }
    void addEveryState(const StEv& se) override {  // :65-84
        StEv cl = cloneStateEvent(se);
        cl->type = CURRENT;
        cl->se[stateId] = nullptr;
        for (int i = stateId; i < (int)cl->se.size(); ++i) cl->se[i] = nullptr;
        Hold st(holder);
        st->newAndEvery.push_back(cl);
        if (partner) {
            cl->se[partner->stateId] = nullptr;
            partner->addToNewAndEvery(cl);
        }
    }
    void resetState() override {  // :87-125
        Hold st(holder);
        if (logicalType == sql::LogicalType::OR || st->pending.size() == partner->pendingSize()) {
            st->pending.clear();
            partner->clearPending();
            if (isStartState && st->newAndEvery.empty()) {
                if (stateType == sql::StateType::SEQUENCE && thisPost->nextEveryStatePre == nullptr &&
                    !thisPost->nextStatePre->pendingEmpty())
                    return;
                init();
            }
        }
    }
    void updateState() override {  // :128-141
        Hold st(holder);
        sortByTime(st->newAndEvery);
        st->pending.splice(st->pending.end(), st->newAndEvery);
        partner->moveAllNewAndEveryToPending();
    }
    Chunk processAndReturn(const SEv& ev) override {  // :143-178
        Chunk ret;
        Hold st(holder);
        auto& lst = st->pending;
        for (auto it = lst.begin(); it != lst.end();) {
            StEv se = *it;
            if (logicalType == sql::LogicalType::OR && se->se[partner->stateId]) {
                it = lst.erase(it);
                continue;
            }
            se->se[stateId] = copyStreamEvent(ev);
            processSE(se);
            if (thisLast->isEventReturned) {
                thisLast->isEventReturned = false;
                ret.add(se);
            }
            if (st->stateChanged) {
                it = lst.erase(it);
            } else {
                se->se[stateId] = nullptr;
                if (stateType == sql::StateType::PATTERN) ++it;
                else it = lst.erase(it);
            }
        }
        return ret;
    }
};

struct LogicalPost : Post {
    sql::LogicalType type = sql::LogicalType::AND;
    LogicalPre* partnerPre = nullptr;
    LogicalPost* partnerPost = nullptr;
    void processSE(StEv se, Chunk& c) override;  // LogicalPostStateProcessor.java:59-87 (after AbsentLogicalPre)
    void setNextStatePreProcessor(PreProc* p) override {
        nextStatePre = p;
        partnerPost->nextStatePre = p;
    }
    void setNextEveryStatePreProcessor(PreProc* p) override {
        nextEveryStatePre = p;
        partnerPost->nextEveryStatePre = p;
    }
};

// ------------------------------------------------------------------------------------------------
// Scheduler (util/Scheduler.java) + AbsentStreamPreStateProcessor
struct SchedState {
    std::deque<int64_t> queue;  // LinkedBlockingQueue (FIFO)
    std::string key;
    bool has_key = false;
    int activeUseCount = 0;
    int64_t seq = 0;  // creation order (live-mode tie break)
    // due index (not reference state, Scheduler::heads): the state's HashMap iteration position = (bucket of its
    // spread hash, newest-inserted first within a bucket -- computeIfAbsent links a new key at the bin's head and
    // resize keeps relative order), with the bucket it was indexed under
    int32_t hash = 0;
    uint64_t stamp = 0, ibucket = 0;
    bool canDestroy() const { return queue.empty(); }
};
using SSP = std::shared_ptr<SchedState>;

struct Scheduler {
    Engine* eng = nullptr;
    PreProc* target = nullptr;  // EntryValveProcessor.setToLast(absentProcessor)
    bool partitioned = false;
    SSP single;
    JHashMap<SSP> map;
    // Due index over the non-empty queues, ordered (head time, map iteration position) -- not reference state. The
    // reference's onTimeChange walks every state of the map per clock advance and keeps, per distinct head time <=
    // now, the first state in iteration order (TreeMultimap with compareTo() == 0); the walk is O(map) per advance,
    // and with the collapse draining one state per due time per advance that was O(keys x events) (C4 at 10^6 keys:
    // hours). The first index entry of each time <= now is the state that walk keeps. ORACLE_SCHED_WALK=1 runs the
    // walk itself (the A/B that pins this index: tests/test_oracle_sched_index.py).
    struct DueKey {
        int64_t t;
        uint64_t bucket, nstamp;
        SchedState* s;
        bool operator<(const DueKey& o) const {
            if (t != o.t) return t < o.t;
            if (bucket != o.bucket) return bucket < o.bucket;
            if (nstamp != o.nstamp) return nstamp < o.nstamp;
            return s < o.s;
        }
    };
    std::set<DueKey> heads;
    size_t idx_cap = 0;  // map.table.size() the index's buckets were computed for
    uint64_t stamps = 0;
    uint64_t bucket_of(const SchedState* st) const {
        return partitioned && !map.table.empty() ? (uint64_t)((map.table.size() - 1) & (uint32_t)st->hash) : 0;
    }
    void idx_sync() {  // a resize moved the states' buckets: re-key the index
        if (map.table.size() == idx_cap) return;
        idx_cap = map.table.size();
        std::vector<SchedState*> all;
        for (const DueKey& d : heads) all.push_back(d.s);
        heads.clear();
        for (SchedState* st : all) {
            st->ibucket = bucket_of(st);
            heads.insert(DueKey{st->queue.front(), st->ibucket, ~st->stamp, st});
        }
    }
    void idx_add(SchedState* st) {
        idx_sync();
        st->ibucket = bucket_of(st);
        heads.insert(DueKey{st->queue.front(), st->ibucket, ~st->stamp, st});
    }
    void idx_del(SchedState* st) {
        idx_sync();
        heads.erase(DueKey{st->queue.front(), st->ibucket, ~st->stamp, st});
    }
    SSP getState();
    void returnState(const SSP& s);
    void notifyAt(int64_t t) {
        SSP s = getState();
        const bool was_empty = s->queue.empty();
        s->queue.push_back(t);
        if (was_empty) idx_add(s.get());
        returnState(s);
    }
    void popHead(const SSP& s) {
        idx_del(s.get());
        s->queue.pop_front();
        if (!s->queue.empty()) idx_add(s.get());
    }
    void sendTimerEvents(const SSP& s);
    void purgeKey(const std::string& k) {  // partition purge: the key's SchedulerState is destroyed
        SSP found;
        map.for_each([&](const std::string& kk, SSP& st) {
            if (kk == k) found = st;
        });
        if (!found) return;
        if (!found->queue.empty()) idx_del(found.get());
        map.remove(k);
    }
    void onTimeChange(int64_t now);  // playback TimeChangeListener
    bool nextDue(int64_t upto, int64_t& t, SSP& st);  // live mode
};

struct Selector;
struct Engine {
    Ctx ctx;
    bool playback = false;
    int64_t lastEventTimestamp = 0;  // TimestampGeneratorImpl (playback clock)
    int64_t liveNow = 0;             // modelled wall clock (live mode)
    int64_t schedSeq = 0;
    std::vector<Scheduler*> schedulers;  // TimeChangeListeners in registration order
    Interner strings;
    int64_t currentTime() const { return playback ? lastEventTimestamp : liveNow; }
    void fireTimer(Scheduler* s, int64_t t, const SSP& st);
};

SSP Scheduler::getState() {
    if (!partitioned) {
        if (!single) { single = std::make_shared<SchedState>(); single->seq = eng->schedSeq++; }
        return single;
    }
    std::string key = eng->ctx.key;
    Engine* e = eng;
    SSP& p = map.computeIfAbsent(key, [&]() {
        auto s = std::make_shared<SchedState>();
        s->key = key;
        s->has_key = true;
        s->seq = e->schedSeq++;
        s->hash = JHashMap<SSP>::spread(key);
        s->stamp = ++stamps;  // insertion order into the map (computeIfAbsent links it at its bin's head)
        return s;
    });
    p->activeUseCount++;
    return p;
}
void Scheduler::returnState(const SSP& s) {
    if (!partitioned) return;
    s->activeUseCount--;
    if (s->activeUseCount == 0 && s->canDestroy()) map.remove(s->key);
}

struct AbsentPost : Post {
    void processSE(StEv se, Chunk& c) override;
};

struct AbsentPre : PreProc {
    int64_t waitingTime = -1;
    Scheduler* scheduler = nullptr;
    bool isAbsent() const override { return true; }
    void updateLastArrivalTime(int64_t ts) override {  // :68-78
        Hold st(holder);
        st->lastScheduledTime = ts + waitingTime;
        scheduler->notifyAt(st->lastScheduledTime);
    }
    void addStateImpl(const StEv& se, const PS& st) override {  // :80-103
        if (!st->active) return;
        if (stateType == sql::StateType::SEQUENCE) {
            st->newAndEvery.clear();
            st->newAndEvery.push_back(se);
        } else {
            st->newAndEvery.push_back(se);
        }
        if (!isStartState) {
            st->lastScheduledTime = se->ts + waitingTime;
            scheduler->notifyAt(st->lastScheduledTime);
        }
    }
    void addEveryState(const StEv& se) override {  // :105-124
        Hold st(holder);
        StEv cl = cloneStateEvent(se);
        cl->type = CURRENT;
        for (int i = stateId; i < (int)cl->se.size(); ++i) cl->se[i] = nullptr;
        st->newAndEvery.push_back(cl);
        st->lastScheduledTime = se->ts + waitingTime;
        scheduler->notifyAt(st->lastScheduledTime);
    }
    void resetState() override {  // :126-148
        Hold st(holder);
        st->pending.clear();
        if (isStartState) {
            if (stateType == sql::StateType::SEQUENCE && thisPost->nextEveryStatePre == nullptr &&
                !thisPost->nextStatePre->pendingEmpty())
                return;
            init();
        }
    }
    void sendEvent(const StEv& se, const PS& st);
    void processTimer(int64_t currentTimeOfChunk) override;  // process(ComplexEventChunk) :151-227
    bool removeOnNoStateChange() const override { return false; }
    Chunk processAndReturn(const SEv& ev) override {  // :257-274
        Hold st(holder);
        if (!st->active) return Chunk();
        Chunk r = PreProc::processAndReturn(ev);
        if (r.first) r = Chunk();
        return r;
    }
    void partitionCreated() override {  // :291-308
        Hold st(holder);
        if (!st->started) {
            st->started = true;
            if (isStartState && waitingTime != -1 && st->active) {
                st->lastScheduledTime = eng->currentTime() + waitingTime;
                scheduler->notifyAt(st->lastScheduledTime);
            }
        }
    }
};

void AbsentPost::processSE(StEv se, Chunk&) {  // AbsentStreamPostStateProcessor.java:36-56
    thisPre->stateChanged();
    StreamEvent* s = se->se[stateId].get();
    se->ts = s->ts;
    isEventReturned = true;
    if (thisPre->isStartState) {
        if (nextEveryStatePre && nextEveryStatePre == thisPre) nextEveryStatePre->addEveryState(se);
    }
    thisPre->updateLastArrivalTime(s->ts);
}

// AbsentLogicalPreStateProcessor.java: one side of `not A [for T] and/or B` (the other side is a LogicalPre or
// another AbsentLogicalPre), with its own scheduler
struct AbsentLogicalPre : LogicalPre {
    int64_t waitingTime = -1;
    Scheduler* scheduler = nullptr;
    bool isAbsent() const override { return true; }
    void updateLastArrivalTime(int64_t ts) override {  // :65-75
        Hold st(holder);
        st->lastArrivalTime = ts;
    }
    void addStateImpl(const StEv& se, const PS& st) override {  // :77-97
        if (!st->active) return;
        LogicalPre::addStateImpl(se, st);
        if (!isStartState && waitingTime != -1) {
            scheduler->notifyAt(se->ts + waitingTime);
            if (partner->isAbsent()) {
                auto* pa = static_cast<AbsentLogicalPre*>(partner);
                pa->scheduler->notifyAt(se->ts + pa->waitingTime);
            }
        }
    }
    void addEveryState(const StEv& se) override {  // :99-118
        StEv cl = cloneStateEvent(se);
        cl->type = CURRENT;
        if (cl->se[stateId]) cl->ts = cl->se[stateId]->ts;  // the timestamp of the last arrived event
        cl->se[stateId] = nullptr;
        cl->se[partner->stateId] = nullptr;
        Hold st(holder);
        st->newAndEvery.push_back(cl);
        partner->addToNewAndEvery(cl);
    }
    bool waitingTimePassed(int64_t currentTime, StateEvent* se) const {  // :220-228
        if (!se->se[stateId]) return currentTime >= se->ts + waitingTime;
        return currentTime >= se->se[stateId]->ts + waitingTime;
    }
    void setActive(bool a) {  // :252-259
        Hold st(holder);
        st->active = a;
    }
    void sendEvent(const StEv& se, const PS& st) {  // :230-250
        if (thisPost->nextProcessor) {
            Chunk one;
            one.add(se);
            thisPost->nextProcessor->process(one);
        }
        if (thisPost->nextStatePre) thisPost->nextStatePre->addState(se);
        if (thisPost->nextEveryStatePre) {
            thisPost->nextEveryStatePre->addEveryState(se);
        } else if (isStartState) {
            st->active = false;
            if (logicalType == sql::LogicalType::OR && partner->isAbsent())
                static_cast<AbsentLogicalPre*>(partner)->setActive(false);
        }
        if (thisPost->callbackPre) thisPost->callbackPre->startStateReset();
    }
    void processTimer(int64_t currentTime) override {  // process(ComplexEventChunk) :121-209
        Hold st(holder);
        if (!st->active) return;
        bool notProcessed = true;
        if (currentTime >= st->lastArrivalTime + waitingTime) {
            if (isStartState && stateType == sql::StateType::SEQUENCE && st->newAndEvery.empty() && st->pending.empty()) {
                StEv se = newStateEvent();
                addState(se);
            } else if (stateType == sql::StateType::SEQUENCE && !st->newAndEvery.empty()) {
                resetState();
            }
            updateState();
            StEv expired;
            std::vector<StEv> ret;
            for (auto it = st->pending.begin(); it != st->pending.end();) {
                StEv se = *it;
                if (isExpired(se.get(), currentTime)) {  // within
                    expired = se;
                    it = st->pending.erase(it);
                    continue;
                }
                if (waitingTimePassed(currentTime, se.get())) {
                    it = st->pending.erase(it);
                    const bool partnerIn = (bool)se->se[partner->stateId];
                    if (logicalType == sql::LogicalType::OR && !partnerIn) {  // OR partner not received
                        se->addEvent(stateId, emptyStreamEvent());
                        ret.push_back(se);
                    } else if (logicalType == sql::LogicalType::AND && partnerIn) {  // AND partner received
                        ret.push_back(se);
                    } else if (logicalType == sql::LogicalType::AND && !partnerIn) {  // let the partner proceed
                        se->addEvent(stateId, emptyStreamEvent());
                    }
                    continue;
                }
                ++it;
            }
            if (expired && withinEveryPre) {
                withinEveryPre->addEveryState(expired);
                withinEveryPre->updateState();
            }
            notProcessed = ret.empty();
            for (auto& se : ret) {
                se->ts = currentTime;
                sendEvent(se, st.s);
            }
            st->lastArrivalTime = 0;
        }
        if (thisPost->nextEveryStatePre || (notProcessed && isStartState)) {  // schedule again
            const int64_t nextBreak = st->lastArrivalTime == 0 ? eng->currentTime() + waitingTime
                                                                : st->lastArrivalTime + waitingTime;
            scheduler->notifyAt(nextBreak);
        }
    }
    Chunk processAndReturn(const SEv& ev) override {  // :262-319 (never returns matches itself)
        Hold st(holder);
        if (!st->active) return Chunk();
        auto& lst = st->pending;
        for (auto it = lst.begin(); it != lst.end();) {
            StEv se = *it;
            if (logicalType == sql::LogicalType::OR && se->se[partner->stateId]) {
                it = lst.erase(it);
                continue;
            }
            SEv curEv = se->se[stateId];
            se->se[stateId] = copyStreamEvent(ev);
            processSE(se);
            if (waitingTime != -1 || (stateType == sql::StateType::SEQUENCE && logicalType == sql::LogicalType::AND &&
                                      thisPost->nextEveryStatePre))
                se->se[stateId] = curEv;  // reset to the original state after processing
            bool removed = false;
            if (thisLast->isEventReturned) {  // passed the filter: no longer an absence candidate
                thisLast->isEventReturned = false;
                it = lst.erase(it);
                removed = true;
                if (stateType == sql::StateType::SEQUENCE) partner->removeFromPending(se);
            }
            if (!st->stateChanged) {
                se->se[stateId] = curEv;
                if (stateType == sql::StateType::SEQUENCE) {
                    if (removed) throw OracleError("IllegalStateException (iterator.remove twice)");
                    it = lst.erase(it);
                    removed = true;
                }
            }
            if (!removed) ++it;
        }
        return Chunk();
    }
    void partitionCreated() override {  // :331-351
        Hold st(holder);
        if (!st->started) {
            st->started = true;
            if (isStartState && waitingTime != -1 && st->active) scheduler->notifyAt(eng->currentTime() + waitingTime);
        }
    }
    bool partnerCanProceed(StateEvent* se) {  // :353-388
        Hold st(holder);
        if (stateType == sql::StateType::SEQUENCE && !thisPost->nextEveryStatePre && st->lastArrivalTime > 0)
            return false;
        if (waitingTime == -1) {
            if (!thisPost->nextEveryStatePre) return !se->se[stateId];  // not received by the absent processor
            if (st->lastArrivalTime > 0) {                                // every
                st->lastArrivalTime = 0;
                init();
                return false;
            }
            return true;
        }
        return (bool)se->se[stateId];
    }
};

void LogicalPost::processSE(StEv se, Chunk& c) {  // LogicalPostStateProcessor.java:59-87
    if (type == sql::LogicalType::AND) {
        const bool proceed = partnerPre->isAbsent() ? static_cast<AbsentLogicalPre*>(partnerPre)->partnerCanProceed(se.get())
                                                    : se->se[partnerPre->stateId] != nullptr;
        if (proceed) Post::processSE(se, c);
        else thisPre->stateChanged();
    } else {
        Post::processSE(se, c);
        if (partnerPost->nextProcessor && thisPre->thisLast == partnerPost) partnerPost->isEventReturned = true;
    }
}

struct AbsentLogicalPost : LogicalPost {  // AbsentLogicalPostStateProcessor.java:37-49
    void processSE(StEv se, Chunk&) override {
        thisPre->stateChanged();
        StreamEvent* s = se->se[stateId].get();
        isEventReturned = true;
        thisPre->updateLastArrivalTime(s->ts);
    }
};

// ------------------------------------------------------------------------------------------------
// selector + outputs
struct OutputRec {
    int kind;  // 0 query callback, 1 stream callback
    std::string name;
    int64_t ts;
    bool expired;
    std::vector<Val> vals;
    std::vector<std::shared_ptr<std::vector<Val>>> lists;
};

struct QueryRt;
struct Selector : Processor {
    struct Attr {
        ExecP ex;
        MultiVarExec* mv = nullptr;
    };
    std::vector<Attr> attrs;
    ExecP having;  // QuerySelector.havingConditionExecutor
    bool currentOn = true, expiredOn = false;
    QueryRt* q = nullptr;
    void process(Chunk& c) override;  // QuerySelector.process -> processNoGroupBy
};

struct AppRt;
struct QueryRt {
    AppRt* app = nullptr;
    std::string name;
    std::string target;
    std::vector<std::unique_ptr<Processor>> owned;
    std::vector<PreProc*> allPre;          // preStateProcessors list (expire order)
    std::vector<PreProc*> startupPre;      // startupPreStateProcessors
    struct Inner;
    Inner* inner = nullptr;
    std::vector<std::unique_ptr<Inner>> inners;
    Selector* selector = nullptr;
    int partition = -1;
    void initPartition();                  // StateStreamRuntime.initPartition :90-97
    void resetAndUpdate();
    // ReturnEventHolder: outputs buffered while a receiver processes one input event
    std::vector<std::vector<StEv>> pendingOut;
    bool buffering = false;
    void sendToCallBacks(std::vector<StEv>& evs);
    std::vector<AggExec*> aggs;            // the selector's aggregators (partition purge cleans their key states)
    void purgeKey(const std::string& key);
};

// InnerStateRuntime tree (query/input/stream/state/runtime/*.java)
struct QueryRt::Inner {
    enum K { STREAM, NEXT, EVERY, LOGICAL, COUNT } k;
    PreProc* first = nullptr;
    Post* last = nullptr;
    Inner* a = nullptr;  // current / inner / rt1
    Inner* b = nullptr;  // next / rt2
    std::vector<std::string> streams;  // single stream runtimes (receiver ids), for setup
    void init() {
        switch (k) {
            case NEXT: a->init(); b->init(); break;
            case EVERY: a->init(); break;
            case LOGICAL: b->init(); a->init(); break;
            default: first->init();
        }
    }
    void reset() {
        switch (k) {
            case NEXT: b->reset(); a->reset(); break;
            case LOGICAL: b->reset(); break;
            default: first->resetState();  // STREAM, COUNT, EVERY (inherits StreamInnerStateRuntime.reset)
        }
    }
    void update() {
        switch (k) {
            case NEXT: a->update(); b->update(); break;
            case LOGICAL: b->update(); break;
            default: first->updateState();
        }
    }
};

void QueryRt::initPartition() {
    inner->init();
    for (PreProc* p : startupPre) p->partitionCreated();
}
void QueryRt::resetAndUpdate() {
    inner->reset();
    inner->update();
}

// receivers
struct Receiver {
    std::string streamId;
    bool multi = false, sequence = false;
    QueryRt* q = nullptr;
    PreProc* next = nullptr;
    std::vector<PreProc*> nextProcessors;
    std::vector<PreProc*> forStream;
    std::vector<int> eventSequence;
    Selector* querySelector = nullptr;
    void setNext(PreProc* p) {
        if (multi) {
            nextProcessors.push_back(p);
            querySelector = dynamic_cast<Selector*>(p->thisPost->nextProcessor);
        } else {
            next = p;
            querySelector = dynamic_cast<Selector*>(p->thisLast->nextProcessor);
        }
    }
    void stabilizeStates(int64_t ts) {
        for (PreProc* p : q->allPre) p->expireEvents(ts);
        if (sequence) {
            q->resetAndUpdate();
        } else if (multi) {
            for (PreProc* p : forStream) p->updateState();
        } else if (!forStream.empty()) {
            forStream[0]->updateState();
        }
    }
    void receive(const SEv& in);
};

void Receiver::receive(const SEv& in) {
    int64_t ts = in->ts;
    stabilizeStates(ts);
    if (multi) {
        // MultiProcessStreamReceiver.receive: every occurrence, in eventSequence order; outputs held
        for (int idx : eventSequence) {
            SEv ev(new StreamEvent());
            ev->ts = in->ts;
            ev->type = in->type;
            ev->data = in->data;
            Chunk c = nextProcessors[idx]->processAndReturn(ev);
            Chunk ret;
            if (c.first) ret.add(c.first);
            c.clear();
            if (querySelector) {
                while (ret.hasNext()) {
                    StEv se = ret.next();
                    ret.remove();
                    q->buffering = true;
                    Chunk one;
                    one.add(se);
                    querySelector->process(one);
                }
            }
        }
        q->buffering = false;
        for (auto& group : q->pendingOut) q->sendToCallBacks(group);
        q->pendingOut.clear();
    } else {
        SEv ev(new StreamEvent());
        ev->ts = in->ts;
        ev->type = in->type;
        ev->data = in->data;
        Chunk c = next->processAndReturn(ev);
        Chunk ret;
        if (c.first) ret.add(c.first);
        c.clear();
        while (ret.hasNext()) {
            StEv se = ret.next();
            ret.remove();
            Chunk one;
            one.add(se);
            if (querySelector) querySelector->process(one);
        }
    }
}

struct PartitionRt {
    int index = 0;
    std::vector<int> queries;
    std::unordered_map<std::string, int64_t> keys;  // PartitionState.partitionKeys: key -> currentTime at its last event
    JavaCHM keyOrder;                                // the same keys in the ConcurrentHashMap's iteration order
    bool purge = false;
    int64_t purge_interval = 0, purge_idle = 0;
    int64_t first_init = INT64_MIN;                 // currentTime of the partition's first initPartition
    struct With {
        int stream;
        ExecP expr;                                           // value partition (null for ranges)
        Type t;
        std::vector<std::pair<ExecP, std::string>> ranges;  // RangePartitionExecutor per range, in order
    };
    std::vector<With> with;
};

struct AppRt {
    Engine eng;
    sql::App app;
    std::vector<std::unique_ptr<QueryRt>> queries;
    std::vector<std::unique_ptr<PartitionRt>> partitions;
    // per stream: ordered subscribers (receivers of top-level queries, partition receivers)
    struct Sub {
        int kind;  // 0 receiver, 1 partition receiver, 2 partition receiver of a stream without a partition key
        Receiver* r = nullptr;
        PartitionRt* p = nullptr;
    };
    std::vector<std::vector<Sub>> subs;
    // per partition, per stream: inner junction receivers
    std::vector<std::unique_ptr<Receiver>> receivers;
    std::map<std::pair<int, int>, std::vector<Receiver*>> innerSubs;  // (partition, stream) -> receivers
    std::vector<OutputRec> outputs;
    bool countOnly = false;
    bool started = false;
    int64_t outCount = 0;
    std::unordered_map<std::string, std::vector<std::string>> streamCallbacks;
    void deliverStream(int stream, const SEv& ev);
    void emitStreamOutput(const std::string& streamId, int64_t ts, bool expired, const std::vector<Val>& vals,
                          const std::vector<std::shared_ptr<std::vector<Val>>>& lists);
};

void QueryRt::purgeKey(const std::string& key) {  // cleanGroupByStates of every StateHolder of the query
    for (PreProc* p : allPre) p->holder.map.erase(key);
    for (Scheduler* s : app->eng.schedulers)
        if (std::find(allPre.begin(), allPre.end(), s->target) != allPre.end()) s->purgeKey(key);
    for (AggExec* a : aggs) a->states.erase(key);
}

void QueryRt::sendToCallBacks(std::vector<StEv>& evs) {
    // OutputRateLimiter.sendToCallBacks :64-108 -> QueryCallback.receiveStreamEvent, InsertIntoStreamCallback
    for (auto& se : evs) {
        if (se->type == EXPIRED || se->type == CURRENT) {
            if (app->countOnly) {
                app->outCount++;
            } else {
                OutputRec r{0, name, se->ts, se->type == EXPIRED, se->out, se->out_list};
                app->outputs.push_back(std::move(r));
            }
        }
    }
    for (auto& se : evs) {
        if (se->type == RESET) continue;
        // expired events are re-typed CURRENT for the insert-into callback
        app->emitStreamOutput(target, se->ts, false, se->out, se->out_list);
    }
}

void Selector::process(Chunk& c) {  // QuerySelector.processNoGroupBy :161-205
    c.reset();
    std::vector<StEv> keep;
    while (c.hasNext()) {
        StEv ev = c.next();
        switch (ev->type) {
            case CURRENT:
            case EXPIRED: {
                for (size_t i = 0; i < attrs.size(); ++i) {
                    if (attrs[i].mv) {
                        ev->out_list[i] = attrs[i].mv->list(ev.get());
                        ev->out[i] = vnull(attrs[i].mv->rt);
                    } else {
                        ev->out[i] = attrs[i].ex->exec(ev.get());
                        ev->out_list[i] = nullptr;
                    }
                }
                if (((ev->type != CURRENT || !currentOn) && (ev->type != EXPIRED || !expiredOn)) ||
                    (having && [&]() { Val h = having->exec(ev.get()); return h.null || !h.b(); }()))
                    c.remove();
                break;
            }
            case RESET:
                break;
            case TIMER:
                c.remove();
                break;
        }
    }
    c.reset();
    std::vector<StEv> out;
    while (c.hasNext()) {
        StEv ev = c.next();
        StEv copy(new StateEvent());  // Event.copyFrom: snapshot the output row now
        copy->ts = ev->ts;
        copy->type = ev->type;
        copy->out = ev->out;
        copy->out_list = ev->out_list;
        out.push_back(copy);
    }
    c.clear();
    if (out.empty()) return;
    if (q->buffering) q->pendingOut.push_back(out);
    else q->sendToCallBacks(out);
}

void AppRt::emitStreamOutput(const std::string& streamId, int64_t ts, bool expired, const std::vector<Val>& vals,
                             const std::vector<std::shared_ptr<std::vector<Val>>>& lists) {
    if (!countOnly) {
        OutputRec r{1, streamId, ts, expired, vals, lists};
        outputs.push_back(std::move(r));
    }
    int si = app.stream_index(streamId);
    if (si >= 0 && si < (int)subs.size() && !subs[si].empty()) {
        SEv ev(new StreamEvent());
        ev->ts = ts;
        ev->data = vals;
        deliverStream(si, ev);
    }
}

// AbsentStreamPreStateProcessor.sendEvent :238-254
void AbsentPre::sendEvent(const StEv& se, const PS& st) {
    if (thisPost->nextProcessor) {
        Chunk one;
        one.add(se);
        thisPost->nextProcessor->process(one);
    }
    if (thisPost->nextStatePre) thisPost->nextStatePre->addState(se);
    if (thisPost->nextEveryStatePre) thisPost->nextEveryStatePre->addEveryState(se);
    else if (isStartState) st->active = false;
    if (thisPost->callbackPre) thisPost->callbackPre->startStateReset();
}

// AbsentStreamPreStateProcessor.process(ComplexEventChunk) :151-227 (TIMER chunk from the scheduler)
void AbsentPre::processTimer(int64_t currentTime) {
    Hold st(holder);
    if (!st->active) return;
    bool notProcessed = true;
    std::vector<StEv> retEvents;
    {
        bool initialize = isStartState && st->newAndEvery.empty() && st->pending.empty();
        if (initialize && stateType == sql::StateType::SEQUENCE && thisPost->nextEveryStatePre == nullptr &&
            st->lastScheduledTime > 0)
            initialize = false;
        if (initialize) {
            StEv se = newStateEvent();
            addState(se);
        } else if (stateType == sql::StateType::SEQUENCE && !st->newAndEvery.empty()) {
            resetState();
        }
        updateState();
        for (auto it = st->pending.begin(); it != st->pending.end();) {
            StEv ev = *it;
            if (isExpired(ev.get(), currentTime)) {
                it = st->pending.erase(it);
                if (withinEveryPre && thisPost->nextEveryStatePre != this) {
                    if (!thisPost->nextEveryStatePre) throw OracleError("NullPointerException in absent expiry");
                    thisPost->nextEveryStatePre->addEveryState(ev);
                }
                continue;
            }
            if ((ev->ts == -1 && currentTime >= st->lastScheduledTime) ||
                (ev->ts != -1 && currentTime >= ev->ts + waitingTime)) {
                it = st->pending.erase(it);
                ev->ts = currentTime;
                retEvents.push_back(ev);
                continue;
            }
            ++it;
        }
        if (withinEveryPre) withinEveryPre->updateState();
    }
    notProcessed = retEvents.empty();
    for (auto& se : retEvents) sendEvent(se, st.s);
    int64_t actualCurrentTime = eng->currentTime();
    if (actualCurrentTime > waitingTime + currentTime) st->lastScheduledTime = actualCurrentTime + waitingTime;
    if (notProcessed && st->lastScheduledTime < currentTime) {
        st->lastScheduledTime = currentTime + waitingTime;
        scheduler->notifyAt(st->lastScheduledTime);
    }
}

void Engine::fireTimer(Scheduler* s, int64_t t, const SSP&) { s->target->processTimer(t); }

// Scheduler.sendTimerEvents :171-209
void Scheduler::sendTimerEvents(const SSP& s) {
    while (!s->queue.empty() && s->queue.front() - eng->currentTime() <= 0) {
        int64_t t = s->queue.front();
        popHead(s);
        eng->fireTimer(this, t, s);
    }
}

// Scheduler TimeChangeListener.onTimeChange :71-103 (playback)
void Scheduler::onTimeChange(int64_t now) {
    if (!partitioned) {
        SSP s = getState();
        if (!s->queue.empty() && s->queue.front() <= now) {
            eng->ctx.has_key = false;
            sendTimerEvents(s);
        }
        return;
    }
    if (heads.empty() || heads.begin()->t > now) return;  // nothing due: the walk below would fire nothing
    static const bool walk = std::getenv("ORACLE_SCHED_WALK") != nullptr;
    if (!walk) {
        // the walk's TreeMultimap holds, per distinct head time <= now, the first state in iteration order: the
        // first index entry of that time. Only those states are used (activeUseCount) and can drain, so they are
        // the only ones returnAllStates can destroy
        idx_sync();
        std::vector<SSP> chosen;
        for (auto it = heads.begin(); it != heads.end() && it->t <= now;) {
            const JHashMap<SSP>::Node* nd = map.find(it->s->key);
            if (!nd) throw OracleError("scheduler due index: a state missing from the map");
            chosen.push_back(nd->val);
            it = heads.lower_bound(DueKey{it->t + 1, 0, 0, nullptr});
        }
        for (auto& st : chosen) st->activeUseCount++;
        for (auto& st : chosen) {
            Ctx saved = eng->ctx;
            eng->ctx.has_key = true;
            eng->ctx.key = st->key;
            sendTimerEvents(st);
            eng->ctx = saved;
        }
        for (auto& st : chosen) {
            st->activeUseCount--;
            if (st->activeUseCount == 0 && st->canDestroy()) map.remove(st->key);
        }
        return;
    }
    // getAllStates (activeUseCount++ on all), TreeMultimap<Long, SchedulerState> with compareTo()==0
    std::vector<SSP> all;
    map.for_each([&](const std::string&, SSP& s) { all.push_back(s); });
    for (auto& s : all) s->activeUseCount++;
    std::map<int64_t, SSP> sorted;
    for (auto& s : all) {
        if (!s->queue.empty() && s->queue.front() <= now) sorted.emplace(s->queue.front(), s);  // first one wins
    }
    for (auto& kv : sorted) {
        Ctx saved = eng->ctx;
        eng->ctx.has_key = true;
        eng->ctx.key = kv.second->key;
        sendTimerEvents(kv.second);
        eng->ctx = saved;
    }
    // returnAllStates: decrement; remove destroyable states in iteration order
    std::vector<std::string> toRemove;
    map.for_each([&](const std::string& k, SSP& s) {
        s->activeUseCount--;
        if (s->activeUseCount == 0 && s->canDestroy()) toRemove.push_back(k);
    });
    for (auto& k : toRemove) map.remove(k);
}

// live mode: earliest due state (notify time, then creation order)
bool Scheduler::nextDue(int64_t upto, int64_t& t, SSP& st) {
    bool found = false;
    auto consider = [&](const SSP& s) {
        if (s->queue.empty()) return;
        int64_t f = s->queue.front();
        if (f > upto) return;
        if (!found || f < t || (f == t && s->seq < st->seq)) { found = true; t = f; st = s; }
    };
    if (!partitioned) {
        if (single) consider(single);
    } else {
        map.for_each([&](const std::string&, SSP& s) { consider(s); });
    }
    return found;
}

// ------------------------------------------------------------------------------------------------
// lowering: StateInputStreamParser + ExpressionParser (subset)
struct MetaEvent {  // MetaStateEvent: one MetaStreamEvent per state slot
    std::vector<const sql::StreamDefinition*> defs;
    std::vector<std::string> refs;
    std::vector<bool> multi;  // count states (multiValue)
};

struct Builder {
    AppRt& rt;
    QueryRt& q;
    const sql::Query& qa;
    MetaEvent meta;
    std::map<std::string, Receiver*> recv;  // processStreamReceiverMap
    bool partitioned;

    bool having_scope = false;           // parsing the having condition: output names resolve first
    std::vector<std::string> out_names;  // the selector's output attributes
    std::vector<Type> out_types;
    Builder(AppRt& r, QueryRt& qq, const sql::Query& a, bool part) : rt(r), q(qq), qa(a), partitioned(part) {}

    template <class T>
    T* own(T* p) {
        q.owned.emplace_back(p);
        return p;
    }

    // ExpressionParser.parseExpression (subset) for a state-event scope
    ExecP expr(const sql::ExprP& e, int currentState, int defaultIdx) {
        using sql::ExprKind;
        switch (e->kind) {
            case ExprKind::CONST: {
                auto c = std::make_unique<ConstExec>();
                c->rt = e->c.type;
                switch (e->c.type) {
                    case Type::INT: c->v = vI((int32_t)e->c.i); break;
                    case Type::LONG: c->v = vL(e->c.i); break;
                    case Type::FLOAT: c->v = vF(e->c.f); break;
                    case Type::DOUBLE: c->v = vD(e->c.d); break;
                    case Type::BOOL: c->v = vB(e->c.i != 0); break;
                    case Type::STRING: c->v = vS(rt.eng.strings.get(e->c.s)); break;
                    default: throw OracleError("unsupported constant");
                }
                return c;
            }
            case ExprKind::VAR: return var(e, currentState, defaultIdx);
            case ExprKind::AND:
            case ExprKind::OR: {
                ExecP a = cond(e->kids[0], currentState, defaultIdx), b = cond(e->kids[1], currentState, defaultIdx);
                if (e->kind == ExprKind::AND) {
                    auto x = std::make_unique<AndExec>();
                    x->l = std::move(a); x->r = std::move(b);
                    return x;
                }
                auto x = std::make_unique<OrExec>();
                x->l = std::move(a); x->r = std::move(b);
                return x;
            }
            case ExprKind::NOT: {
                auto x = std::make_unique<NotExec>();
                x->x = cond(e->kids[0], currentState, defaultIdx);
                return x;
            }
            case ExprKind::CMP: {
                ExecP a = expr(e->kids[0], currentState, defaultIdx), b = expr(e->kids[1], currentState, defaultIdx);
                Type lt = a->rt, rtp = b->rt;
                bool eq = e->cmp == sql::CmpOp::EQ || e->cmp == sql::CmpOp::NE;
                if (lt == Type::STRING || rtp == Type::STRING) {
                    if (!(lt == Type::STRING && rtp == Type::STRING) || !eq)
                        throw OracleError("OperationNotSupportedException: string compare");
                } else if (lt == Type::BOOL || rtp == Type::BOOL) {
                    if (!(lt == Type::BOOL && rtp == Type::BOOL) || !eq)
                        throw OracleError("OperationNotSupportedException: bool compare");
                } else if (lt == Type::OBJECT || rtp == Type::OBJECT) {
                    throw OracleError("OperationNotSupportedException: object compare");
                }
                auto x = std::make_unique<CmpExec>();
                x->op = e->cmp;
                x->lt = lt;
                x->rtp = rtp;
                x->l = std::move(a);
                x->r = std::move(b);
                return x;
            }
            case ExprKind::ADD: case ExprKind::SUB: case ExprKind::MUL: case ExprKind::DIV: case ExprKind::MOD: {
                ExecP a = expr(e->kids[0], currentState, defaultIdx), b = expr(e->kids[1], currentState, defaultIdx);
                auto x = std::make_unique<MathExec>();
                if (a->rt == Type::DOUBLE || b->rt == Type::DOUBLE) x->rt = Type::DOUBLE;
                else if (a->rt == Type::FLOAT || b->rt == Type::FLOAT) x->rt = Type::FLOAT;
                else if (a->rt == Type::LONG || b->rt == Type::LONG) x->rt = Type::LONG;
                else if (a->rt == Type::INT || b->rt == Type::INT) x->rt = Type::INT;
                else throw OracleError("ArithmeticException");
                if (!sql::is_numeric(a->rt) || !sql::is_numeric(b->rt)) throw OracleError("ArithmeticException");
                x->k = e->kind;
                x->l = std::move(a);
                x->r = std::move(b);
                return x;
            }
            case ExprKind::IS_NULL: {
                auto x = std::make_unique<IsNullExec>();
                x->x = expr(e->kids[0], currentState, defaultIdx);
                return x;
            }
            case ExprKind::IS_NULL_STREAM: {
                auto x = std::make_unique<IsNullStreamExec>();
                int idx = defaultIdx;
                if (e->has_index) idx = e->index <= sql::IDX_LAST ? e->index + 1 : e->index;
                int chain = -1;
                for (size_t i = 0; i < meta.refs.size(); ++i) {
                    if ((meta.refs[i].empty() && meta.defs[i]->id == e->stream_ref) || meta.refs[i] == e->stream_ref) {
                        chain = (int)i;
                        if (!meta.refs[i].empty() && currentState > -1 && !meta.refs[currentState].empty() &&
                            e->has_index && e->index <= sql::IDX_LAST && e->stream_ref == meta.refs[currentState])
                            idx = e->index;
                        break;
                    }
                }
                if (chain < 0) throw OracleError("stream reference not found for is null");
                x->chain = chain;
                x->idx = idx;
                return x;
            }
            case ExprKind::FUNC: return func(e, currentState, defaultIdx);
            default:
                throw OracleError("OperationNotSupportedException: expression kind not supported");
        }
    }
    // ExpressionParser.parseExpression AttributeFunction: core functions (executor/function) and, in the selector
    // / having scope only, attribute aggregators (query/selector/attribute/aggregator)
    ExecP func(const sql::ExprP& e, int cs, int di) {
        const std::string& n = e->fn_name;
        auto bad = [&](const std::string& m) { return OracleError("SiddhiAppValidationException: " + n + "(): " + m); };
        if (!e->fn_ns.empty())
            throw OracleError("OperationNotSupportedException: function '" + e->fn_ns + ":" + n + "' is not supported");
        std::vector<ExecP> args;
        for (auto& k : e->kids) args.push_back(expr(k, cs, di));
        auto same_types = [&]() {
            for (auto& a : args)
                if (a->rt != args[0]->rt) throw bad("all parameters should be of the same type");
        };
        if (n == "ifThenElse") {
            if (args.size() != 3) throw bad("required 3 arguments");
            if (args[0]->rt != Type::BOOL) throw bad("the condition must be bool");
            if (args[1]->rt != args[2]->rt) throw bad("then / else types differ");
            auto x = std::make_unique<IfThenElseExec>();
            x->rt = args[1]->rt;
            x->c = std::move(args[0]); x->a = std::move(args[1]); x->b = std::move(args[2]);
            return x;
        }
        if (n == "coalesce" || n == "default") {
            if (args.empty()) throw bad("needs arguments");
            if (n == "default" && (args.size() != 2 || e->kids[1]->kind != sql::ExprKind::CONST))
                throw bad("takes (attribute, constant default)");
            same_types();
            auto x = std::make_unique<CoalesceExec>();
            x->rt = args[0]->rt;
            x->xs = std::move(args);
            return x;
        }
        static const std::pair<const char*, Type> inst[] = {
            {"instanceOfBoolean", Type::BOOL}, {"instanceOfDouble", Type::DOUBLE}, {"instanceOfFloat", Type::FLOAT},
            {"instanceOfInteger", Type::INT},  {"instanceOfLong", Type::LONG},     {"instanceOfString", Type::STRING}};
        for (auto& p : inst)
            if (n == p.first) {
                if (args.size() != 1) throw bad("required 1 argument");
                auto x = std::make_unique<InstanceOfExec>();
                x->rt = Type::BOOL;
                x->target = p.second;
                x->x = std::move(args[0]);
                return x;
            }
        if (n == "maximum" || n == "minimum") {
            if (args.empty()) throw bad("needs arguments");
            for (auto& a : args)
                if (!sql::is_numeric(a->rt)) throw bad("numeric parameters required");
            same_types();
            auto x = std::make_unique<MaxMinExec>();
            x->rt = args[0]->rt;
            x->is_max = n == "maximum";
            x->xs = std::move(args);
            return x;
        }
        static const std::pair<const char*, AggExec::K> aggs[] = {
            {"count", AggExec::COUNT}, {"sum", AggExec::SUM}, {"avg", AggExec::AVG}, {"min", AggExec::MIN},
            {"max", AggExec::MAX}, {"minForever", AggExec::MIN}, {"maxForever", AggExec::MAX}};
        for (auto& p : aggs)
            if (n == p.first) {
                if (cs != -1) throw OracleError("SiddhiAppCreationException: aggregator " + n + "() outside the selector");
                auto x = std::make_unique<AggExec>();
                x->k = p.second;
                x->ctx = &rt.eng.ctx;
                x->partitioned = partitioned;
                q.aggs.push_back(x.get());
                if (x->k == AggExec::COUNT) {
                    if (!args.empty()) throw bad("takes no arguments");
                    x->rt = Type::LONG;
                    return x;
                }
                if (args.size() != 1 || !sql::is_numeric(args[0]->rt))
                    throw OracleError("OperationNotSupportedException: " + n + "() needs one numeric argument");
                x->at = args[0]->rt;
                x->arg = std::move(args[0]);
                if (x->k == AggExec::SUM) x->rt = (x->at == Type::INT || x->at == Type::LONG) ? Type::LONG : Type::DOUBLE;
                else if (x->k == AggExec::AVG) x->rt = Type::DOUBLE;
                else x->rt = x->at;
                return x;
            }
        throw OracleError("OperationNotSupportedException: function '" + n + "' is not supported");
    }
    ExecP cond(const sql::ExprP& e, int cs, int di) {
        ExecP x = expr(e, cs, di);
        if (x->rt != Type::BOOL) throw OracleError("condition must be bool");
        return x;
    }
    // ExpressionParser.parseVariable, MetaStateEvent branch :1302-1438
    ExecP var(const sql::ExprP& e, int currentState, int defaultIdx, bool* multiOut = nullptr) {
        if (having_scope && e->stream_ref.empty()) {  // :1310-1318: the output definition first
            for (size_t j = 0; j < out_names.size(); ++j)
                if (out_names[j] == e->attr) {
                    auto x = std::make_unique<OutVarExec>();
                    x->j = (int)j;
                    x->rt = out_types[j];
                    return x;
                }
        }
        int idx = defaultIdx;
        if (e->has_index) idx = e->index <= sql::IDX_LAST ? e->index + 1 : e->index;
        int chain = -1;
        Type type = Type::OBJECT;
        bool multiValue = false;
        if (e->stream_ref.empty()) {
            if (currentState == -1) {
                bool found = false;
                for (size_t i = 0; i < meta.defs.size(); ++i) {
                    int ai = meta.defs[i]->index_of(e->attr);
                    if (ai < 0) continue;
                    if (found) throw OracleError("SiddhiAppValidationException: ambiguous attribute '" + e->attr + "'");
                    found = true;
                    chain = (int)i;
                    type = meta.defs[i]->attrs[ai].type;
                }
            } else {
                int ai = meta.defs[currentState]->index_of(e->attr);
                if (ai < 0) throw OracleError("SiddhiAppValidationException: attribute '" + e->attr + "' not found");
                chain = currentState;
                type = meta.defs[currentState]->attrs[ai].type;
            }
        } else {
            for (size_t i = 0; i < meta.defs.size(); ++i) {
                if (meta.refs[i].empty()) {
                    if (meta.defs[i]->id == e->stream_ref) {
                        int ai = meta.defs[i]->index_of(e->attr);
                        if (ai < 0) throw OracleError("attribute not found");
                        type = meta.defs[i]->attrs[ai].type;
                        chain = (int)i;
                        break;
                    }
                } else if (meta.refs[i] == e->stream_ref) {
                    int ai = meta.defs[i]->index_of(e->attr);
                    if (ai < 0) throw OracleError("attribute not found");
                    type = meta.defs[i]->attrs[ai].type;
                    chain = (int)i;
                    if (currentState > -1 && !meta.refs[currentState].empty() && e->has_index &&
                        e->index <= sql::IDX_LAST) {
                        if (e->stream_ref == meta.refs[currentState]) idx = e->index;
                    } else if (currentState == -1 && !e->has_index) {
                        multiValue = meta.multi[i];
                    }
                    break;
                }
            }
        }
        if (chain < 0) throw OracleError("SiddhiAppValidationException: no stream reference for '" + e->attr + "'");
        if (multiOut) *multiOut = multiValue;
        if (multiValue) {
            auto m = std::make_unique<MultiVarExec>();
            m->rt = type;
            m->chain = chain;
            m->attr = meta.defs[chain]->index_of(e->attr);
            return m;
        }
        auto v = std::make_unique<VarExec>();
        v->rt = type;
        v->chain = chain;
        v->idx = idx;
        v->attr = meta.defs[chain]->index_of(e->attr);
        return v;
    }

    Receiver* receiver(const std::string& sid) { return recv.at(sid); }

    // StateInputStreamParser.parse :148-408
    QueryRt::Inner* parse(const sql::StateP& el, PreProc* pre, Post* post, bool multiValue,
                          std::vector<PreProc*>& preList, bool isStart) {
        using sql::StateKind;
        auto mkInner = [&](QueryRt::Inner::K k) {
            q.inners.emplace_back(new QueryRt::Inner());
            q.inners.back()->k = k;
            return q.inners.back().get();
        };
        if (el->kind == StateKind::STREAM || el->kind == StateKind::ABSENT) {
            const sql::StreamDefinition* def = rt.app.stream(el->stream_id);
            if (!def) throw OracleError("SiddhiAppCreationException: stream '" + el->stream_id + "' is not defined");
            meta.defs.push_back(def);
            meta.refs.push_back(el->ref);
            meta.multi.push_back(multiValue);
            int stateIndex = (int)meta.defs.size() - 1;
            // filters: SingleInputStreamParser -> FilterProcessor(parseExpression(..., stateIndex, CURRENT))
            Processor* chainHead = nullptr;
            Processor* chainTail = nullptr;
            for (auto& f : el->filters) {
                auto* fp = own(new FilterProc());
                fp->cond = expr(f, stateIndex, sql::IDX_CURRENT);
                if (fp->cond->rt != Type::BOOL) throw OracleError("filter must be bool");
                if (!chainHead) chainHead = fp;
                else chainTail->setToLast(fp);
                chainTail = fp;
            }
            if (!pre) {
                if (el->kind == StateKind::ABSENT) {
                    auto* ap = own(new AbsentPre());
                    ap->kind = PreKind::ABSENT;
                    ap->waitingTime = el->waiting_ms;
                    q.startupPre.push_back(ap);
                    auto* sch = new Scheduler();
                    sch->eng = &rt.eng;
                    sch->target = ap;
                    sch->partitioned = partitioned;
                    rt.eng.schedulers.push_back(sch);
                    ap->scheduler = sch;
                    pre = ap;
                } else {
                    pre = own(new PreProc());
                }
                pre->eng = &rt.eng;
                pre->stateType = qa.state_type;
                pre->holder.ctx = &rt.eng.ctx;
                pre->holder.partitioned = partitioned;
            }
            pre->stateId = stateIndex;
            pre->isStartState = isStart;
            pre->nattrs = (int)def->attrs.size();
            pre->nextProcessor = chainHead;  // setNextProcessor(singleStreamRuntime.getProcessorChain())
            if (!post) {
                post = el->kind == StateKind::ABSENT ? (Post*)own(new AbsentPost()) : own(new Post());
            }
            post->stateId = stateIndex;
            if (pre->nextProcessor) pre->nextProcessor->setToLast(post);
            else pre->nextProcessor = post;
            post->thisPre = pre;
            pre->thisPost = post;
            pre->thisLast = post;
            auto* in = mkInner(QueryRt::Inner::STREAM);
            in->first = pre;
            in->last = post;
            in->streams.push_back(el->stream_id);
            preList.push_back(pre);
            return in;
        }
        if (el->kind == StateKind::NEXT) {
            auto* cur = parse(el->kids[0], pre, post, multiValue, preList, isStart);
            auto* nxt = parse(el->kids[1], pre, post, multiValue, preList, false);
            cur->last->setNextStatePreProcessor(nxt->first);
            auto* in = mkInner(QueryRt::Inner::NEXT);
            in->a = cur;
            in->b = nxt;
            in->first = cur->first;
            in->last = nxt->last;
            in->streams = cur->streams;
            in->streams.insert(in->streams.end(), nxt->streams.begin(), nxt->streams.end());
            return in;
        }
        if (el->kind == StateKind::EVERY) {
            std::vector<PreProc*> withinEvery;
            auto* inner = parse(el->kids[0], pre, post, multiValue, withinEvery, isStart);
            auto* in = mkInner(QueryRt::Inner::EVERY);
            in->a = inner;
            in->first = inner->first;
            in->last = inner->last;
            in->streams = inner->streams;
            in->last->setNextEveryStatePreProcessor(in->first);
            for (PreProc* p : withinEvery) p->withinEveryPre = in->first;
            preList.insert(preList.end(), withinEvery.begin(), withinEvery.end());
            return in;
        }
        if (el->kind == StateKind::LOGICAL) {
            // StateInputStreamParser.parse :289-378: an absent element becomes an AbsentLogicalPreStateProcessor
            // with its own scheduler (element 1's created first), registered as a startup processor
            auto mkPre = [&](const sql::StateP& kid) -> LogicalPre* {
                if (kid->kind != StateKind::ABSENT) return own(new LogicalPre());
                auto* ap = own(new AbsentLogicalPre());
                ap->waitingTime = kid->waiting_ms;
                q.startupPre.push_back(ap);
                auto* sch = new Scheduler();
                sch->eng = &rt.eng;
                sch->target = ap;
                sch->partitioned = partitioned;
                rt.eng.schedulers.push_back(sch);
                ap->scheduler = sch;
                return ap;
            };
            LogicalPre* p1 = mkPre(el->kids[0]);
            LogicalPre* p2 = mkPre(el->kids[1]);
            for (LogicalPre* p : {p1, p2}) {
                p->kind = PreKind::LOGICAL;
                p->logicalType = el->logical;
                p->eng = &rt.eng;
                p->stateType = qa.state_type;
                p->holder.ctx = &rt.eng.ctx;
                p->holder.partitioned = partitioned;
            }
            LogicalPost* o1 = el->kids[0]->kind == StateKind::ABSENT ? own(new AbsentLogicalPost()) : own(new LogicalPost());
            LogicalPost* o2 = el->kids[1]->kind == StateKind::ABSENT ? own(new AbsentLogicalPost()) : own(new LogicalPost());
            o1->type = o2->type = el->logical;
            o1->partnerPre = p2;
            o2->partnerPre = p1;
            o1->partnerPost = o2;
            o2->partnerPost = o1;
            p1->partner = p2;
            p2->partner = p1;
            auto* in2 = parse(el->kids[1], p2, o2, multiValue, preList, isStart);
            auto* in1 = parse(el->kids[0], p1, o1, multiValue, preList, isStart);
            auto* in = mkInner(QueryRt::Inner::LOGICAL);
            in->a = in1;
            in->b = in2;
            in->first = in1->first;
            in->last = in2->last;
            in->streams = in2->streams;
            in->streams.insert(in->streams.end(), in1->streams.begin(), in1->streams.end());
            return in;
        }
        if (el->kind == StateKind::COUNT) {
            int mn = el->min_count == sql::COUNT_ANY ? 0 : el->min_count;
            int mx = el->max_count == sql::COUNT_ANY ? INT32_MAX : el->max_count;
            auto* cp = own(new CountPre());
            cp->kind = PreKind::COUNT;
            cp->minCount = mn;
            cp->maxCount = mx;
            cp->eng = &rt.eng;
            cp->stateType = qa.state_type;
            cp->holder.ctx = &rt.eng.ctx;
            cp->holder.partitioned = partitioned;
            auto* co = own(new CountPost());
            co->minCount = mn;
            co->maxCount = mx;
            cp->countPost = co;
            auto* inner = parse(el->kids[0], cp, co, true, preList, isStart);
            auto* in = mkInner(QueryRt::Inner::COUNT);
            in->first = inner->first;
            in->last = inner->last;
            in->streams = inner->streams;
            return in;
        }
        throw OracleError("OperationNotSupportedException");
    }

    // StreamInnerStateRuntime.setup / Next / Logical (setup order)
    void setup(QueryRt::Inner* in) {
        switch (in->k) {
            case QueryRt::Inner::NEXT: setup(in->a); setup(in->b); break;
            case QueryRt::Inner::EVERY: setup(in->a); break;
            case QueryRt::Inner::LOGICAL: setup(in->b); setup(in->a); break;
            default: {
                Receiver* r = receiver(in->streams[0]);
                r->setNext(in->first);
                r->forStream.push_back(in->first);
            }
        }
    }

    void build() {
        // receivers by stream count (StateInputStreamParser :91-110); stream ids in first-appearance order
        std::vector<std::string> ids;
        std::map<std::string, int> counts;
        std::function<void(const sql::StateP&)> walk = [&](const sql::StateP& e) {
            if (e->kind == sql::StateKind::STREAM || e->kind == sql::StateKind::ABSENT) {
                if (!counts.count(e->stream_id)) ids.push_back(e->stream_id);
                counts[e->stream_id]++;
            }
            for (auto& k : e->kids) walk(k);
        };
        walk(qa.root);
        for (auto& sid : ids) {
            auto* r = new Receiver();
            rt.receivers.emplace_back(r);
            r->streamId = sid;
            r->q = &q;
            r->multi = counts[sid] > 1;
            r->sequence = qa.state_type == sql::StateType::SEQUENCE;
            int n = counts[sid];
            for (int i = 0; i < n; ++i) r->eventSequence.push_back(i);
            if (r->multi) std::reverse(r->eventSequence.begin(), r->eventSequence.end());
            recv[sid] = r;
        }
        std::vector<PreProc*> preList;
        q.inner = parse(qa.root, nullptr, nullptr, false, preList, true);
        q.allPre = preList;
        int nst = (int)meta.defs.size();
        // selector (SelectorParser: UNKNOWN_STATE, default index 0)
        auto* sel = own(new Selector());
        sel->q = &q;
        sel->currentOn = qa.out_type != sql::OutputEventType::EXPIRED;
        sel->expiredOn = qa.out_type != sql::OutputEventType::CURRENT;
        // select *: every attribute of every state's stream, unqualified (SelectorParser.getAttributeProcessors
        // :182-209; a name in two streams is a DuplicateAttributeException)
        std::vector<sql::OutputAttribute> sel_list = qa.select;
        if (qa.select_all) {
            sel_list.clear();
            for (auto* d : meta.defs)
                for (auto& at : d->attrs) {
                    for (auto& o : sel_list)
                        if (o.rename == at.name) throw OracleError("DuplicateAttributeException: '" + at.name + "'");
                    sql::OutputAttribute o;
                    o.rename = at.name;
                    o.expr = std::make_shared<sql::Expr>();
                    o.expr->kind = sql::ExprKind::VAR;
                    o.expr->attr = at.name;
                    sel_list.push_back(o);
                }
        }
        out_names.clear();
        for (auto& oa : sel_list) out_names.push_back(oa.rename);
        for (auto& oa : sel_list) {
            Selector::Attr a;
            bool mv = false;
            if (oa.expr->kind == sql::ExprKind::VAR) {
                a.ex = var(oa.expr, -1, 0, &mv);
                if (mv) a.mv = static_cast<MultiVarExec*>(a.ex.get());
            } else {
                a.ex = expr(oa.expr, -1, 0);
            }
            sel->attrs.push_back(std::move(a));
        }
        for (auto& a : sel->attrs) out_types.push_back(a.ex->rt);
        if (qa.having) {  // HAVING_STATE, default chain index 0 (SelectorParser.generateHavingExecutor)
            having_scope = true;
            sel->having = cond(qa.having, -1, 0);
            having_scope = false;
        }
        q.selector = sel;
        for (PreProc* p : preList) {
            p->nstates = nst;
            p->noutputs = (int)sel->attrs.size();
        }
        if (qa.has_within) {
            std::vector<int> startIds;
            for (PreProc* p : preList)
                if (p->isStartState) startIds.push_back(p->stateId);
            for (PreProc* p : preList) {
                p->startStateIds = startIds;
                p->withinTime = qa.within_ms;
            }
        }
        q.inner->first->thisLast = q.inner->last;
        // StateStreamRuntime.setCommonProcessor: setQuerySelector then setup
        setQuerySelector(q.inner, sel);
        setup(q.inner);
    }
    void setQuerySelector(QueryRt::Inner* in, Selector* s) {
        switch (in->k) {
            case QueryRt::Inner::NEXT: setQuerySelector(in->b, s); break;
            case QueryRt::Inner::EVERY: setQuerySelector(in->a, s); break;
            case QueryRt::Inner::LOGICAL: setQuerySelector(in->b, s); setQuerySelector(in->a, s); break;
            default: in->last->setNextProcessor(s);
        }
    }
};

void AppRt::deliverStream(int stream, const SEv& ev) {
    Ctx outer = eng.ctx;
    for (auto& sub : subs[stream]) {
        if (sub.kind == 0) {
            eng.ctx.has_key = false;
            eng.ctx.key.clear();
            sub.r->receive(ev);
            eng.ctx = outer;
        } else if (sub.kind == 2) {
            // PartitionStreamReceiver.send(ComplexEvent) (:274-283): a stream with no partition executor goes to
            // every key of getPartitionKeys() (PartitionRuntimeImpl.java:404-407), in that HashSet's order; no
            // initPartition, no partitionKeys.put (the keys' purge clocks do not move)
            auto it = innerSubs.find({sub.p->index, stream});
            if (it == innerSubs.end()) continue;
            for (const std::string& key : sub.p->keyOrder.hashset_order()) {
                eng.ctx.has_key = true;
                eng.ctx.key = key;
                for (Receiver* r : it->second) r->receive(ev);
            }
            eng.ctx = outer;
        } else {
            PartitionRt* p = sub.p;
            for (auto& w : p->with) {
                if (w.stream != stream) continue;
                StEv holder(new StateEvent());
                holder->se.resize(1);
                holder->se[0] = ev;
                std::vector<std::string> keys;
                if (!w.expr) {  // RangePartitionExecutor.execute: the label when the condition holds, else null
                    for (auto& r : w.ranges) {
                        Val c = r.first->exec(holder.get());
                        if (!c.null && c.b()) keys.push_back(r.second);
                    }
                } else {  // ValuePartitionExecutor: expr.execute(event).toString(); null -> dropped
                    Val v = w.expr->exec(holder.get());
                    if (v.null) continue;
                    std::string key;
                    switch ((Type)v.t) {
                        case Type::STRING: key = eng.strings.strs[(uint32_t)v.raw]; break;
                        case Type::INT: key = std::to_string(v.i()); break;
                        case Type::LONG: key = std::to_string(v.l()); break;
                        case Type::FLOAT: key = java_real_to_string(v.f(), true); break;
                        case Type::DOUBLE: key = java_real_to_string(v.d(), false); break;
                        case Type::BOOL: key = v.b() ? "true" : "false"; break;
                        default: break;
                    }
                    keys.push_back(key);
                }
                for (const std::string& key : keys) {  // PartitionStreamReceiver.send(key, event) per executor
                Ctx saved = eng.ctx;
                eng.ctx.has_key = true;
                eng.ctx.key = key;
                const int64_t now = eng.currentTime();
                if (p->purge) {
                    // @purge (PartitionRuntimeImpl.initPartition :368-401): a task every `interval` ms destroys the
                    // states of keys idle for more than idle.period (by currentTime). The reference runs it on a
                    // scheduled executor in wall-clock time -- and registers one more such task on every
                    // initPartition call, so passes are near-continuous once the first interval has elapsed.
                    // Modelling assumption: a pass at every clock reading from first_init + interval on; a key's
                    // state is destroyed before its next event when that event's clock exceeds its last activity
                    // by idle.period (equivalent for every key with no pending timer).
                    auto it = p->keys.find(key);
                    if (it != p->keys.end() && p->first_init != INT64_MIN && now >= p->first_init + p->purge_interval &&
                        it->second + p->purge_idle < now) {
                        p->keys.erase(it);
                        p->keyOrder.remove(key);
                        for (int qi : p->queries) queries[qi]->purgeKey(key);
                    }
                }
                if (!p->keys.count(key)) {  // PartitionRuntimeImpl.initPartition
                    for (int qi : p->queries) queries[qi]->initPartition();
                    if (p->first_init == INT64_MIN) p->first_init = now;
                }
                p->keys[key] = now;
                p->keyOrder.put(key);  // partitionKeys.put: a new key, or a walk along its bin (treeifyBin)
                auto it = innerSubs.find({p->index, stream});
                if (it != innerSubs.end())
                    for (Receiver* r : it->second) r->receive(ev);
                eng.ctx = saved;
                }
            }
        }
    }
}

}  // namespace orc

// ------------------------------------------------------------------------------------------------
// C API
using namespace orc;

struct orc_engine {
    AppRt rt;
};

static thread_local std::string g_err;

extern "C" const char* orc_last_error(void) { return g_err.c_str(); }

static void build_app(orc_engine* e, const char* text) {
    AppRt& rt = e->rt;
    rt.app = sql::parse_app(text);
    rt.eng.playback = rt.app.playback;
    rt.subs.resize(rt.app.streams.size());
    for (size_t pi = 0; pi < rt.app.partitions.size(); ++pi) {
        auto* p = new PartitionRt();
        p->index = (int)pi;
        rt.partitions.emplace_back(p);
        p->queries = rt.app.partitions[pi].queries;
        p->purge = rt.app.partitions[pi].purge;
        p->purge_interval = rt.app.partitions[pi].purge_interval_ms;
        p->purge_idle = rt.app.partitions[pi].purge_idle_ms;
    }
    for (size_t qi = 0; qi < rt.app.queries.size(); ++qi) {
        const sql::Query& qa = rt.app.queries[qi];
        if (qa.target_inner) throw OracleError("unsupported: inner (#) streams");
        auto* q = new QueryRt();
        rt.queries.emplace_back(q);
        q->app = &rt;
        q->name = qa.name;
        q->target = qa.target;
        q->partition = qa.partition_index;
        Builder b(rt, *q, qa, qa.partition_index >= 0);
        b.build();
        // subscribe receivers (SiddhiAppRuntimeBuilder.addQuery / PartitionRuntime inner junctions)
        for (auto& kv : b.recv) {
            int si = rt.app.stream_index(kv.first);
            if (si < 0) throw OracleError("stream not defined: " + kv.first);
            if (qa.partition_index < 0) {
                AppRt::Sub s;
                s.kind = 0;
                s.r = kv.second;
                rt.subs[si].push_back(s);
            } else {
                rt.innerSubs[{qa.partition_index, si}].push_back(kv.second);
            }
        }
        // output stream: define it implicitly if not declared
        if (!rt.app.stream(qa.target)) {
            sql::StreamDefinition d;
            d.id = qa.target;
            rt.app.streams.push_back(d);
            rt.subs.resize(rt.app.streams.size());
        }
    }
    // partition receivers subscribe to the outer junctions
    for (size_t pi = 0; pi < rt.app.partitions.size(); ++pi) {
        auto& pa = rt.app.partitions[pi];
        PartitionRt* p = rt.partitions[pi].get();
        std::vector<int> streamsSeen;
        for (auto& w : pa.with) {
            int si = rt.app.stream_index(w.stream_id);
            if (si < 0) throw OracleError("partition stream not defined: " + w.stream_id);
            PartitionRt::With pw;
            pw.stream = si;
            // expression over the single stream event (slot 0)
            QueryRt tmpq;
            sql::Query dummy;
            Builder b(rt, tmpq, dummy, false);
            b.meta.defs.push_back(&rt.app.streams[si]);
            b.meta.refs.push_back("");
            b.meta.multi.push_back(false);
            if (w.ranges.empty()) {
                pw.expr = b.expr(w.expr, 0, sql::IDX_CURRENT);
                pw.t = pw.expr->rt;
            } else {
                for (auto& r : w.ranges) pw.ranges.push_back({b.cond(r.first, 0, sql::IDX_CURRENT), r.second});
                pw.t = Type::STRING;
            }
            p->with.push_back(std::move(pw));
            if (std::find(streamsSeen.begin(), streamsSeen.end(), si) == streamsSeen.end()) {
                streamsSeen.push_back(si);
                AppRt::Sub s;
                s.kind = 1;
                s.p = p;
                rt.subs[si].push_back(s);
            }
        }
        // streams of the partition's queries without a partition key: PartitionRuntimeImpl.addPartitionReceiver
        // (:290-304) subscribes a PartitionStreamReceiver with no executors, which broadcasts (kind 2)
        for (auto& kv : rt.innerSubs)
            if (kv.first.first == (int)pi && std::find(streamsSeen.begin(), streamsSeen.end(), kv.first.second) == streamsSeen.end()) {
                AppRt::Sub s;
                s.kind = 2;
                s.p = p;
                rt.subs[kv.first.second].push_back(s);
            }
    }
}

// SiddhiAppRuntime.start (core/SiddhiAppRuntimeImpl.java:440): initPartition of the top-level queries
static void start_app(orc_engine* e, int64_t start_ts) {
    AppRt& rt = e->rt;
    if (rt.started) return;
    rt.started = true;
    if (!rt.eng.playback) rt.eng.liveNow = start_ts;
    for (auto& q : rt.queries)
        if (q->partition < 0) q->initPartition();
}

extern "C" int orc_start(orc_engine* e, int64_t start_ts) {
    try {
        start_app(e, start_ts);
        return 0;
    } catch (const std::exception& ex) {
        g_err = ex.what();
        return -1;
    }
}

extern "C" orc_engine* orc_create(const char* app, char* err, int errlen) {
    auto* e = new orc_engine();
    try {
        build_app(e, app);
        return e;
    } catch (const std::exception& ex) {
        g_err = ex.what();
        if (err && errlen > 0) std::snprintf(err, errlen, "%s", ex.what());
        delete e;
        return nullptr;
    }
}

extern "C" void orc_destroy(orc_engine* e) {
    if (!e) return;
    for (auto* s : e->rt.eng.schedulers) delete s;
    delete e;
}

extern "C" int orc_stream_index(orc_engine* e, const char* sid) { return e->rt.app.stream_index(sid); }
extern "C" int orc_num_attrs(orc_engine* e, int s) { return (int)e->rt.app.streams[s].attrs.size(); }
extern "C" int orc_attr_type(orc_engine* e, int s, int a) { return (int)e->rt.app.streams[s].attrs[a].type; }
extern "C" uint32_t orc_intern(orc_engine* e, const char* s) { return e->rt.eng.strings.get(s); }
extern "C" const char* orc_string(orc_engine* e, uint32_t id) {
    if (id >= e->rt.eng.strings.strs.size()) return nullptr;
    return e->rt.eng.strings.strs[id].c_str();
}

// ---- state dump: every StateHolder's snapshot() map of the pattern processors -------------------------------
// StreamPreState.snapshot() (StreamPreStateProcessor.java:450-459) + CountStreamPreState (CountPreStateProcessor
// .java:206-212), AbsentStreamPreState (AbsentStreamPreStateProcessor.java:328-334), LogicalStreamPreState of an
// absent side (AbsentLogicalPreStateProcessor.java:407-413), as JSON:
//   {"queries":[{"name":..,"states":{"<partition key>":{"<stateId>":{"FirstEvent":..,"PendingStateEventList":[SE..],
//     "NewAndEveryStateEventList":[SE..],"Initialized":..,"Started":.., +subclass fields}}}}]}
//   SE = {"ts":..,"type":..,"events":[null | [{"ts":..,"data":[v..]} ..] per position]}
// States a holder would destroy on return (canDestroy) are left out, as are keys left with none: the dump shows
// what a snapshot taken between two events holds. Values: integers, reals as "%.17g" of the double (strings
// "NaN" / "Infinity" / "-Infinity"), booleans, strings; null.
static void dump_str(std::string& o, const std::string& s) {
    o += '"';
    for (unsigned char c : s) {
        if (c == '"' || c == '\\') {
            o += '\\';
            o += (char)c;
        } else if (c < 0x20) {
            char b[8];
            std::snprintf(b, sizeof b, "\\u%04x", c);
            o += b;
        } else {
            o += (char)c;
        }
    }
    o += '"';
}
static void dump_real(std::string& o, double x) {
    if (x != x) { o += "\"NaN\""; return; }
    if (std::isinf(x)) { o += x > 0 ? "\"Infinity\"" : "\"-Infinity\""; return; }
    char b[40];
    std::snprintf(b, sizeof b, "%.17g", x);
    o += b;
}
static void dump_val(std::string& o, const Val& v, const Interner& S) {
    if (v.null) { o += "null"; return; }
    switch ((Type)v.t) {
        case Type::INT: o += std::to_string(v.i()); break;
        case Type::LONG: o += std::to_string(v.l()); break;
        case Type::FLOAT: dump_real(o, (double)v.f()); break;
        case Type::DOUBLE: dump_real(o, v.d()); break;
        case Type::BOOL: o += v.b() ? "true" : "false"; break;
        default: dump_str(o, v.raw >= 0 && (size_t)v.raw < S.strs.size() ? S.strs[(size_t)v.raw] : std::string()); break;
    }
}
static void dump_se(std::string& o, const StateEvent* s, const Interner& S) {
    if (!s) { o += "null"; return; }
    o += "{\"ts\":" + std::to_string(s->ts) + ",\"type\":" + std::to_string((int)s->type) + ",\"events\":[";
    for (size_t p = 0; p < s->se.size(); ++p) {
        if (p) o += ',';
        const StreamEvent* e = s->se[p].get();
        if (!e) { o += "null"; continue; }
        o += '[';
        for (bool first = true; e; e = e->next.get(), first = false) {
            if (!first) o += ',';
            o += "{\"ts\":" + std::to_string(e->ts) + ",\"data\":[";
            for (size_t j = 0; j < e->data.size(); ++j) {
                if (j) o += ',';
                dump_val(o, e->data[j], S);
            }
            o += "]}";
        }
        o += ']';
    }
    o += "]}";
}
static void dump_list(std::string& o, const std::list<StEv>& l, const Interner& S) {
    o += '[';
    bool first = true;
    for (const StEv& s : l) {
        if (!first) o += ',';
        first = false;
        dump_se(o, s.get(), S);
    }
    o += ']';
}
static void dump_state(std::string& o, const PreProc* p, const PreState& s, const Interner& S) {
    o += "{\"FirstEvent\":";
    dump_se(o, s.cur.first.get(), S);
    o += ",\"PendingStateEventList\":";
    dump_list(o, s.pending, S);
    o += ",\"NewAndEveryStateEventList\":";
    dump_list(o, s.newAndEvery, S);
    o += std::string(",\"Initialized\":") + (s.initialized ? "true" : "false");
    o += std::string(",\"Started\":") + (s.started ? "true" : "false");
    if (p->kind == PreKind::COUNT) {
        o += std::string(",\"SuccessCondition\":") + (s.successCondition ? "true" : "false");
        o += std::string(",\"StartStateReset\":") + (s.startStateReset ? "true" : "false");
    } else if (dynamic_cast<const AbsentLogicalPre*>(p)) {
        o += std::string(",\"IsActive\":") + (s.active ? "true" : "false");
        o += ",\"LastArrivalTime\":" + std::to_string(s.lastArrivalTime);
    } else if (p->kind == PreKind::ABSENT) {
        o += std::string(",\"IsActive\":") + (s.active ? "true" : "false");
        o += ",\"LastScheduledTime\":" + std::to_string(s.lastScheduledTime);
    }
    o += '}';
}

static thread_local std::string g_dump;

extern "C" const char* orc_state_dump(orc_engine* e) {
    try {
        const Interner& S = e->rt.eng.strings;
        std::string& o = g_dump;
        o = "{\"queries\":[";
        for (size_t qi = 0; qi < e->rt.queries.size(); ++qi) {
            const QueryRt& q = *e->rt.queries[qi];
            if (qi) o += ',';
            o += "{\"name\":";
            dump_str(o, q.name);
            o += ",\"states\":{";
            std::vector<const PreProc*> pres(q.allPre.begin(), q.allPre.end());
            std::sort(pres.begin(), pres.end(), [](const PreProc* a, const PreProc* b) { return a->stateId < b->stateId; });
            // key -> (stateId -> state)
            std::map<std::string, std::vector<std::pair<int, const PreState*>>> keys;
            for (const PreProc* p : pres) {
                const PreStateHolder& h = p->holder;
                if (!h.partitioned) {
                    if (h.single && !h.single->canDestroy()) keys[""].push_back({p->stateId, h.single.get()});
                } else {
                    for (const auto& kv : h.map)
                        if (kv.second && !kv.second->canDestroy()) keys[kv.first].push_back({p->stateId, kv.second.get()});
                }
            }
            bool fk = true;
            for (const auto& kv : keys) {
                if (!fk) o += ',';
                fk = false;
                dump_str(o, kv.first);
                o += ":{";
                for (size_t i = 0; i < kv.second.size(); ++i) {
                    if (i) o += ',';
                    o += '"' + std::to_string(kv.second[i].first) + "\":";
                    const PreProc* p = nullptr;
                    for (const PreProc* x : pres)
                        if (x->stateId == kv.second[i].first) p = x;
                    dump_state(o, p, *kv.second[i].second, S);
                }
                o += '}';
            }
            o += "}}";
        }
        o += "]}";
        return o.c_str();
    } catch (const std::exception& ex) {
        g_err = ex.what();
        return nullptr;
    }
}

static void live_fire_until(orc_engine* e, int64_t t) {
    Engine& g = e->rt.eng;
    while (true) {
        int64_t best = 0;
        SSP bs;
        Scheduler* bsch = nullptr;
        for (Scheduler* s : g.schedulers) {
            int64_t tt;
            SSP st;
            if (s->nextDue(t, tt, st)) {
                if (!bsch || tt < best || (tt == best && st->seq < bs->seq)) { best = tt; bs = st; bsch = s; }
            }
        }
        if (!bsch) break;
        if (best > g.liveNow) g.liveNow = best;
        Ctx saved = g.ctx;
        g.ctx.has_key = bs->has_key;
        g.ctx.key = bs->key;
        bs->activeUseCount++;
        bsch->sendTimerEvents(bs);
        g.ctx = saved;
        bs->activeUseCount--;
        if (bsch->partitioned && bs->activeUseCount == 0 && bs->canDestroy()) bsch->map.remove(bs->key);
    }
    if (t > g.liveNow) g.liveNow = t;
}

static void advance(orc_engine* e, int64_t ts) {
    Engine& g = e->rt.eng;
    if (g.playback) {
        // TimestampGeneratorImpl.setCurrentTimestamp :105-122
        if (ts >= g.lastEventTimestamp) {
            g.lastEventTimestamp = ts;
            for (Scheduler* s : g.schedulers) s->onTimeChange(ts);
        }
    } else {
        live_fire_until(e, ts);
    }
}

// mode 0: InputHandler.send(ts, data); mode 1: InputHandler.send(data) (timestamp = currentTime()); mode 2: one
// event of an InputHandler.send(Event[]) (:85-95): the caller moved the clock once for the array (orc_advance_time
// to the last event's timestamp), the event itself does not move it.
// now: the modelled wall clock (live mode); ignored in playback.
static void send_one(orc_engine* e, int stream, int64_t ts, int64_t now, int mode, const int64_t* slots,
                     const uint8_t* nulls) {
    AppRt& rt = e->rt;
    Engine& g = rt.eng;
    start_app(e, g.playback ? ts : now);
    if (g.playback) {
        if (mode == 0) advance(e, ts);
        else if (mode == 1) ts = g.currentTime();
    } else {
        if (mode != 2) advance(e, now);
        if (mode == 1) ts = now;
    }
    const auto& def = rt.app.streams[stream];
    SEv ev(new StreamEvent());
    ev->ts = ts;
    ev->data.resize(def.attrs.size());
    for (size_t a = 0; a < def.attrs.size(); ++a) {
        Val v;
        v.t = (uint8_t)def.attrs[a].type;
        v.null = nulls && nulls[a];
        v.raw = v.null ? 0 : slots[a];
        if (def.attrs[a].type == Type::INT) v.raw = (int32_t)v.raw;
        if (def.attrs[a].type == Type::FLOAT) v.raw = (uint32_t)v.raw;
        ev->data[a] = v;
    }
    rt.deliverStream(stream, ev);
}

extern "C" int orc_send(orc_engine* e, int stream, int64_t ts, const int64_t* slots, const uint8_t* nulls) {
    try {
        send_one(e, stream, ts, ts, 0, slots, nulls);
        return 0;
    } catch (const std::exception& ex) {
        g_err = ex.what();
        return -1;
    }
}

extern "C" int orc_send_ex(orc_engine* e, int stream, int64_t ts, int64_t now, int mode, const int64_t* slots,
                           const uint8_t* nulls) {
    try {
        send_one(e, stream, ts, now, mode, slots, nulls);
        return 0;
    } catch (const std::exception& ex) {
        g_err = ex.what();
        return -1;
    }
}

extern "C" int orc_send_batch(orc_engine* e, int64_t n, const int32_t* stream, const int64_t* ts,
                              const int64_t* offsets, const int64_t* slots, const uint8_t* nulls) {
    try {
        for (int64_t i = 0; i < n; ++i)
            send_one(e, stream[i], ts[i], ts[i], 0, slots + offsets[i], nulls ? nulls + offsets[i] : nullptr);
        return 0;
    } catch (const std::exception& ex) {
        g_err = ex.what();
        return -1;
    }
}

extern "C" int orc_advance_time(orc_engine* e, int64_t ts) {
    try {
        start_app(e, ts);
        advance(e, ts);
        return 0;
    } catch (const std::exception& ex) {
        g_err = ex.what();
        return -1;
    }
}

extern "C" int64_t orc_num_outputs(orc_engine* e) { return (int64_t)e->rt.outputs.size(); }
extern "C" int orc_output(orc_engine* e, int64_t i, int* kind, const char** name, int64_t* ts, int* expired, int* nvals) {
    const OutputRec& r = e->rt.outputs[i];
    *kind = r.kind;
    *name = r.name.c_str();
    *ts = r.ts;
    *expired = r.expired;
    *nvals = (int)r.vals.size();
    return 0;
}
extern "C" int orc_output_value(orc_engine* e, int64_t i, int j, int64_t* slot, int* is_null) {
    const OutputRec& r = e->rt.outputs[i];
    if (j < (int)r.lists.size() && r.lists[j]) {
        *slot = 0;
        *is_null = 0;
        return 7;
    }
    *slot = r.vals[j].raw;
    *is_null = r.vals[j].null;
    return r.vals[j].t;
}
extern "C" int orc_output_list_len(orc_engine* e, int64_t i, int j) {
    const OutputRec& r = e->rt.outputs[i];
    return (j < (int)r.lists.size() && r.lists[j]) ? (int)r.lists[j]->size() : -1;
}
extern "C" int orc_output_list_item(orc_engine* e, int64_t i, int j, int k, int64_t* slot, int* is_null) {
    const Val& v = (*e->rt.outputs[i].lists[j])[k];
    *slot = v.raw;
    *is_null = v.null;
    return v.t;
}
extern "C" void orc_clear_outputs(orc_engine* e) { e->rt.outputs.clear(); }
extern "C" void orc_count_only(orc_engine* e, int on) { e->rt.countOnly = on != 0; }
extern "C" int64_t orc_output_count(orc_engine* e) { return e->rt.outCount; }

// bulk export of the query-callback outputs (kind 0, non-list values) in delivery order: ts[n], vals[n][nv]
// (row-major), nulls[n][nv]; returns the number of rows written (at most cap)
extern "C" int64_t orc_export_query_outputs(orc_engine* e, int64_t cap, int nv, int64_t* ts, int64_t* vals,
                                            uint8_t* nulls) {
    int64_t k = 0;
    for (const OutputRec& r : e->rt.outputs) {
        if (r.kind != 0 || r.expired) continue;
        if (k >= cap) break;
        ts[k] = r.ts;
        for (int j = 0; j < nv; ++j) {
            const bool ok = j < (int)r.vals.size();
            vals[k * nv + j] = ok ? r.vals[j].raw : 0;
            nulls[k * nv + j] = ok ? r.vals[j].null : 1;
        }
        ++k;
    }
    return k;
}
