// One partition key's NFA (nfa.h, the same code the gfx950 kernel runs) executed on the host, for two callers:
//   * the scheduler simulation (sched.h): when the reference's global scheduler orders a key's timer fires
//     differently from the key's own device run in a way that changes its result, the simulation replays that key
//     from its batch-start state with the exact order of events and fires, and keeps stepping it in lockstep;
//   * spilled keys (engine.cpp): a key that outgrows the device arena's 4096 partial matches continues on the host
//     in an arena of 32-bit indices (KeyRunT<int32_t>) that doubles whenever the key needs more.
#pragma once
#include <stdint.h>

#include <vector>

#include "nfa.h"

namespace sdg {

// a host run's match records (same record layout as the device's)
struct KeyOut {
    uint32_t key = 0;
    std::vector<int64_t> o_ts, o_vals, o_seq, o_sub;
    std::vector<uint32_t> o_nulls, o_key;
    unsigned long long count = 0;
};

template <class IX>
struct KeyRunT : KeyOut {
    std::vector<uint8_t> arena;                      // batch-start state, then the run's state
    // the key's rows in this batch (time order), as the sorted view holds them
    std::vector<int64_t> ts;
    std::vector<uint8_t> qs;
    std::vector<uint32_t> pos;                       // batch position of each row
    std::vector<uint32_t> vrank;                     // the rows' delivery ranks (range / broadcast rows), or empty
    std::vector<std::vector<uint8_t>> cols, nulls;   // per physical column: raw values / null flags
    bool has_qs = false;
    std::vector<nfa::SchedLog> log;
    unsigned long long lcount = 0;
    size_t lread = 0;

    void start(const Plan* P, const Instr* code, const int64_t* consts, const nfa::Layout& L, const nfa::TimerIn& T,
               int64_t seq_base, const nfa::PurgeIn* purge = nullptr) {
        P_ = P;
        if (purge) c_.purge = *purge;
        n_out_ = P->n_out;
        ncols_ = P->n_cols;
        c_.P = P;
        c_.code = code;
        c_.consts = consts;
        c_.L = L;
        c_.base = arena.data();
        stk_.assign(STACK, 0);
        c_.stk = stk_.data();
        c_.stride = 1;
        c_.emit_count = &count;
        c_.flags = flags_;
        c_.key = key;
        c_.emit_round = nullptr;
        c_.round = 0;
        c_.T = T;
        c_.T.log_count = &lcount;
        c_.fires = nullptr;
        c_.nfires = 0;  // explicit (empty) list: the simulation calls fire() itself
        reserve(1024);
        for (int k = 0; k < ncols_; ++k) {
            cptr_[k] = cols[k].data();
            nptr_[k] = nulls[k].empty() ? nullptr : nulls[k].data();
        }
        ev_ = nfa::KeyEvents{ts.data(), has_qs ? qs.data() : nullptr, pos.data(), cptr_, nptr_, 0, (int64_t)ts.size(),
                             seq_base, 0, vrank.empty() ? nullptr : vrank.data()};
        need_init_ = nfa::key_begin(c_, ev_);
        p_ = 0;
    }
    // rows with position < g (the fires before them were stepped already)
    bool rows_before(int64_t g) {
        while (p_ < (int64_t)ts.size() && (int64_t)pos[p_] < g) {
            reserve(0);
            if (!nfa::key_row(c_, ev_, p_++, need_init_)) return false;
        }
        return true;
    }
    bool row_at(int64_t g) { return rows_before(g + 1); }
    void fire(int sch, uint32_t g, int64_t clock) {
        reserve(0);
        c_.fire(sch, g, clock);
    }
    void finish(const nfa::TimerIn& T) {
        if (T.G > 0) c_.clock = T.clk[T.G - 1];
    }
    bool overflow() { return c_.ovf() || flags_[0] || flags_[5]; }
    bool arena_overflow() { return c_.ovf(); }
    bool output_overflow() const { return flags_[0] != 0; }
    unsigned long long emitted() const { return count; }  // records the run asked for (> the sink on overflow)
    int64_t slack = 4096;  // free output slots kept before each step (one event can complete many partials)
    int64_t next_row_pos() const { return p_ < (int64_t)ts.size() ? (int64_t)pos[p_] : -1; }
    int64_t purge_last() const { return c_.purge.last; }  // the key's last activity after the replay (@purge)

   private:
    const Plan* P_ = nullptr;
    int n_out_ = 0, ncols_ = 0;
    nfa::CtxT<true, IX> c_;
    nfa::KeyEvents ev_{};
    const void* cptr_[MAX_COLS] = {};
    const uint8_t* nptr_[MAX_COLS] = {};
    std::vector<int64_t> stk_;
    int flags_[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    int64_t p_ = 0;
    bool need_init_ = false;
    // keep room for a step's worth of outputs and log records (the sinks are plain host vectors)
    void reserve(int64_t min_cap) {
        int64_t cap = (int64_t)o_ts.size();
        if (cap - (int64_t)count < slack || cap < min_cap) {
            const int64_t nc = std::max<int64_t>({min_cap, 2 * cap, (int64_t)count + 2 * slack});
            std::vector<int64_t> v((size_t)std::max(n_out_, 1) * nc);
            for (int j = 0; j < n_out_; ++j)
                for (unsigned long long i = 0; i < count; ++i) v[(size_t)j * nc + i] = o_vals[(size_t)j * cap + i];
            o_vals.swap(v);
            o_ts.resize(nc);
            o_seq.resize(nc);
            o_sub.resize(nc);
            o_nulls.resize(nc);
            o_key.resize(nc);
            c_.emit_ts = o_ts.data();
            c_.emit_vals = o_vals.data();
            c_.emit_nulls = o_nulls.data();
            c_.emit_seq = o_seq.data();
            c_.emit_sub = o_sub.data();
            c_.emit_key = o_key.data();
            c_.emit_cap = nc;
        }
        if ((int64_t)log.size() - (int64_t)lcount < 4096) {
            log.resize(std::max<size_t>(2 * log.size(), lcount + 8192));
            c_.T.log = log.data();
            c_.T.log_cap = (int64_t)log.size();
        }
    }
};
using KeyRun = KeyRunT<int16_t>;

}  // namespace sdg
