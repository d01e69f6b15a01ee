// Host check of crypto-recommendation_amd/csrc/kmseg.h: the segmented
// evaluation of the reference's fp64 chain s_i = fl(s_{i-1} + x_i)
// (update.hpp:52-56) against the plain chain, bit for bit, with the same
// window / pair / record-capacity structure as update.hip's kernels and the
// approximate prefix sums they predict binades from -- also with those
// predictions deliberately perturbed (every misprediction must fall back to
// real adds, never change the result).
// Built and run by tests/test_lib_cpu.py (CPU). Exit code 0 = all equal.
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>
#include <vector>

#include "../crypto-recommendation_amd/csrc/kmseg.h"

using namespace lshkm;

static volatile double g_sink;
static double chain(double s, const std::vector<double>& x) {
    for (double v : x) { s = s + v; g_sink = s; }
    return s;
}

struct Stats { long recs = 0, fails = 0, dense = 0, steps = 0; };

// The update.hip pipeline for one chain: pairs = the chain cut at window
// boundaries (first pair starts at offset off0 of its window); pass A: pair
// sums; pass B: approximate pair start sums; pass C: segments per pair (up to
// KS_R records, else dense); pass D: composition.
static double segmented(double s0, const std::vector<double>& x, int off0, double noise, std::mt19937_64& rng,
                        Stats& st) {
    const int n = (int)x.size();
    std::vector<int> pb;                      // pair starts
    for (int p = 0; p < n;) {
        pb.push_back(p);
        const int o = (p == 0) ? off0 : 0;
        p += KS_W - o;
    }
    pb.push_back(n);
    const int np = (int)pb.size() - 1;
    std::vector<double> psum(np), sin(np);
    for (int q = 0; q < np; q++) {            // A
        double t = 0.0;
        for (int p = pb[q]; p < std::min(pb[q + 1], n); p++) t += x[p];
        psum[q] = t;
    }
    double run = s0;                          // B
    for (int q = 0; q < np; q++) { sin[q] = run; run += psum[q]; }
    std::normal_distribution<double> nd(0.0, 1.0);
    std::vector<std::vector<KsRec>> recs(np);
    std::vector<int> cnt(np);
    for (int q = 0; q < np; q++) {            // C
        const int beg = pb[q], end = std::min(pb[q + 1], n);
        const int obase = (q == 0) ? off0 : 0;
        double sa = sin[q];
        KsSeg g;
        bool open = false;
        int nr = 0;
        auto emit = [&](const KsSeg& gg) {
            if (nr < KS_R) recs[q].push_back(ks_record(gg));
            nr++;
        };
        for (int p = beg; p < end; p++) {
            sa += x[p];
            double pred = sa;
            if (noise > 0.0) pred = sa * (1.0 + noise * nd(rng));
            ks_feed(g, open, x[p], pred, obase + (p - beg), emit);
        }
        if (open) emit(g);
        cnt[q] = nr;
    }
    double s = s0;                            // D
    for (int q = 0; q < np; q++) {
        const int beg = pb[q], end = std::min(pb[q + 1], n);
        const int obase = (q == 0) ? off0 : 0;
        st.steps += end - beg;
        if (cnt[q] > KS_R) {
            st.dense++;
            for (int p = beg; p < end; p++) s = s + x[p];
            continue;
        }
        for (const KsRec& r : recs[q]) {
            st.recs++;
            if (!ks_apply(s, r)) {
                st.fails++;
                for (int o = ks_rec_a(r) + 1; o <= ks_rec_b(r); o++) s = s + x[beg + (o - obase)];
            }
        }
    }
    return s;
}

static bool same(double a, double b) { return memcmp(&a, &b, 8) == 0; }

int main(int argc, char** argv) {
    const int reps = argc > 1 ? atoi(argv[1]) : 40;
    std::mt19937_64 rng(12345);
    std::normal_distribution<double> nd(0.0, 1.0);
    std::uniform_real_distribution<double> ud(0.0, 1.0);
    long bad = 0, total = 0;
    Stats st;
    for (int rep = 0; rep < reps; rep++) {
        for (int fam = 0; fam < 9; fam++) {
            const int n = 1 + (int)(ud(rng) * (fam < 2 ? 70000 : 6000));
            std::vector<double> x(n);
            double s0 = 0.0;
            for (int i = 0; i < n; i++) {
                switch (fam) {
                case 0: x[i] = nd(rng); break;                                          // random walk
                case 1: x[i] = 0.3 + nd(rng); break;                                    // drift
                case 2: x[i] = (double)(2 * (int)(ud(rng) * 8) + 1); s0 = 0x1p53; break;  // ties at G = 2
                case 3: x[i] = ldexp(nd(rng), (int)(ud(rng) * 60) - 30); break;         // wide range
                case 4: x[i] = ldexp(std::round(nd(rng) * 64), -7); s0 = ldexp(1.0, 50); break;  // dyadic, ties
                case 5: x[i] = nd(rng) * 1e-310; break;                                 // subnormal walk
                case 6: x[i] = (i % 997 == 5) ? (i % 2 ? INFINITY : NAN) : nd(rng); break;
                case 7: x[i] = (i % 1500 == 7) ? 1.5e308 : nd(rng) * 1e300; break;      // overflow to inf
                case 8: x[i] = (i % 2 ? 1.0 : -1.0) * ldexp(1.0 + ud(rng), (int)(ud(rng) * 4)); s0 = -0.0; break;
                }
            }
            if (fam == 0 && rep % 3 == 1) s0 = 123.456;
            const double want = chain(s0, x);
            for (int pert = 0; pert < 3; pert++) {
                const double noise = pert == 0 ? 0.0 : (pert == 1 ? 1e-9 : 1e-3);
                const int off0 = (int)(ud(rng) * KS_W);
                const double got = segmented(s0, x, off0, noise, rng, st);
                total++;
                if (!same(got, want) && !(std::isnan(got) && std::isnan(want))) {
                    if (bad < 10) printf("MISMATCH fam=%d n=%d pert=%d: %.17g vs %.17g\n", fam, n, pert, got, want);
                    bad++;
                }
            }
        }
    }
    printf("chains=%ld bad=%ld steps=%ld records=%ld (%.4f/step) fallbacks=%ld dense_pairs=%ld\n", total, bad, st.steps,
           st.recs, (double)st.recs / (double)st.steps, st.fails, st.dense);
    return bad ? 1 : 0;
}
