// Replays the host scheduler simulation (siddhi_amd/csrc/engine/sched.cpp, optimistic pass) on inputs dumped by
// the test emulator (SDG_SIM_DUMP=path python3 scripts/emu_prof.py c4 ...), timed, with an optional SIGPROF
// sample of program counters (argv[3]) for addr2line. Benchmark infrastructure, CPU only:
//   hipcc -std=c++17 -O2 -g -x hip --cuda-host-only scripts/simbench.cpp siddhi_amd/csrc/engine/sched.cpp -o /tmp/simbench
#include <signal.h>
#include <sys/time.h>
#include <ucontext.h>

#include <chrono>
#include <cstdio>
#include <cstring>
#include <vector>

#include "../siddhi_amd/csrc/engine/sched.h"

using namespace sdg;

static std::vector<uintptr_t> g_s(1 << 22);
static volatile size_t g_n = 0;
static void on_prof(int, siginfo_t*, void* uc) {
    if (g_n < g_s.size()) g_s[g_n++] = (uintptr_t)((ucontext_t*)uc)->uc_mcontext.gregs[REG_RIP];
}

template <class T>
static void rv(FILE* f, std::vector<T>& v) {
    uint64_t m = 0;
    if (std::fread(&m, 8, 1, f) != 1) throw 1;
    v.resize(m);
    if (m && std::fread(v.data(), sizeof(T), m, f) != m) throw 1;
}

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    FILE* f = std::fopen(argv[1], "rb");
    int64_t hdr[6];
    if (!f || std::fread(hdr, 8, 6, f) != 6) return 3;
    BatchClock bc;
    bc.G = hdr[0];
    bc.clock0 = hdr[1];
    std::vector<nfa::SchedLog> logs;
    std::vector<int32_t> key_hash;
    std::vector<uint32_t> seg_b, seg_e, gpos;
    rv(f, bc.clk); rv(f, bc.adv); rv(f, bc.nadv); rv(f, logs); rv(f, key_hash); rv(f, seg_b); rv(f, seg_e); rv(f, gpos);
    std::fclose(f);
    KeyRows kr;
    kr.seg_b = seg_b.data();
    kr.seg_e = seg_e.data();
    kr.K = (int64_t)seg_b.size();
    kr.orig = gpos.data();
    kr.n = hdr[5];
    const int reps = argc > 2 ? std::atoi(argv[2]) : 3;
    if (argc > 3) {
        struct sigaction sa;
        std::memset(&sa, 0, sizeof sa);
        sa.sa_sigaction = on_prof;
        sa.sa_flags = SA_SIGINFO | SA_RESTART;
        sigaction(SIGPROF, &sa, nullptr);
        itimerval tv{{0, 500}, {0, 500}};
        setitimer(ITIMER_PROF, &tv, nullptr);
    }
    double best = 1e30;
    size_t nre = 0;
    int64_t nf = 0;
    for (int r = 0; r < reps; ++r) {
        SchedSim sim;
        sim.setup((int)hdr[2], hdr[3] != 0, hdr[4] != 0);
        SchedSim::Result res;
        auto t0 = std::chrono::steady_clock::now();
        sim.simulate(bc, logs, key_hash, kr, [](uint32_t) -> KeyRun* { return nullptr; }, res, true);
        const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
        best = std::min(best, ms);
        nre = res.reordered.size();
        nf = res.n_fires;
    }
    if (argc > 3) {
        itimerval tv{{0, 0}, {0, 0}};
        setitimer(ITIMER_PROF, &tv, nullptr);
        FILE* o = std::fopen(argv[3], "w");
        for (size_t i = 0; i < g_n; ++i) std::fprintf(o, "0x%lx\n", (unsigned long)g_s[i]);
        std::fclose(o);
    }
    std::printf("logs %zu fires %lld reordered %zu: optimistic pass best %.1f ms of %d\n", logs.size(), (long long)nf,
                nre, best, reps);
    return 0;
}
