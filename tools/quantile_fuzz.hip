// Host-side check that vigra_quantiles_cross (crossing search) and
// vigra_quantiles (keypoint walk) give bit-identical quantiles.
// build: hipcc -O2 -std=c++17 --offload-arch=gfx950 tools/quantile_fuzz.hip -o /tmp/qfuzz && /tmp/qfuzz
#include "../cluster_tools_amd/csrc/ctg_reduce.hip"
#include <cstdio>
#include <cstring>
#include <random>

int main() {
    std::mt19937_64 rng(12345);
    long bad = 0, n = 0;
    for (int it = 0; it < 2000000; ++it) {
        uint32_t h[ctg::NSLOTS] = {0};
        const int mode = it % 7;
        const int nz = 1 + (int)(rng() % (mode == 0 ? 1 : mode == 1 ? 3 : 42));
        for (int j = 0; j < nz; ++j) {
            int slot = (int)(rng() % ctg::NSLOTS);
            if (mode == 2 && (slot == 0 || slot == ctg::NSLOTS - 1)) slot = 1 + (int)(rng() % ctg::NBINS);
            h[slot] += 1 + (uint32_t)(rng() % (mode == 3 ? 3 : 2000));
        }
        uint64_t cnt = 0;
        int lo = -1, hi = -1;
        for (int s = 0; s < ctg::NSLOTS; ++s) {
            cnt += h[s];
            if (h[s]) { if (lo < 0) lo = s; hi = s; }
        }
        std::uniform_real_distribution<double> U(0.0, 1.0);
        auto in_slot = [&](int s, bool low) {
            if (s == 0) return -U(rng) * 3.0;
            if (s == ctg::NSLOTS - 1) return 1.0 + 1e-6 + U(rng) * 3.0;
            const int k = s - 1;
            const int r = (int)(rng() % 4);
            if (r == 0) return (double)(float)(k / 40.0);                      // bin edge
            if (r == 1 && k == ctg::NBINS - 1 && !low) return 1.0;            // top edge maps into bin 39
            return (double)(float)((k + U(rng)) / 40.0);
        };
        double vmin = in_slot(lo, true), vmax = in_slot(hi, false);
        if (lo == hi && vmin > vmax) std::swap(vmin, vmax);
        const double scale = (mode == 6) ? 40.0 / 255.0 : 40.0, offset = (mode == 6) ? 0.0 : 0.0;
        if (mode == 6) { vmin *= 255.0; vmax *= 255.0; }
        double a[5] = {0, 0, 0, 0, 0}, b[5] = {0, 0, 0, 0, 0};
        ctg::vigra_quantiles(h, (double)cnt, vmin, vmax, scale, offset, a);
        ctg::vigra_quantiles_cross(h, (double)cnt, vmin, vmax, scale, offset, b);
        ++n;
        if (std::memcmp(a, b, sizeof a) != 0) {
            if (bad < 10) {
                std::printf("mismatch it=%d mode=%d cnt=%llu vmin=%.17g vmax=%.17g lo=%d hi=%d\n", it, mode,
                            (unsigned long long)cnt, vmin, vmax, lo, hi);
                for (int q = 0; q < 5; ++q) std::printf("  q%d walk=%.17g cross=%.17g\n", q, a[q], b[q]);
            }
            ++bad;
        }
    }
    std::printf("%ld / %ld mismatches\n", bad, n);
    return bad != 0;
}
