// Synthetic PreAccept stream generator.  Host code; deterministic from seed.
//
// Txn i (0-based; TxnId order == index order):
//   TxnId(epoch=1, hlc=1_000_000+i, flags=kind<<1|domain, node=1+(i mod node_mod))
//   (packing: Timestamp.java:81-89 msb = epoch<<15 | hlc>>>48, lsb = hlc<<16 | flags;
//    flags: TxnId.java:124-157)
//   key txns: kind = Write w.p. write_frac else Read; k distinct key ordinals drawn
//   Zipf(s) over the keyspace (rank -> ordinal through a seeded permutation), sorted
//   (Keys.of sorts and de-duplicates: primitives/Keys.java:129-131).
//   range txns: kind Read/Write 50/50, domain Range; 1..ranges_max ranges (s, s+len],
//   len ~ U[1, range_len_max], normalised like Ranges.of (sort + merge strictly overlapping:
//   AbstractRanges.java:696-782, MERGE_OVERLAPPING).
#include "../../include/accord_deps.h"

#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <vector>

namespace {

struct SplitMix64 {
    uint64_t s;
    explicit SplitMix64(uint64_t seed) : s(seed) {}
    uint64_t next() {
        uint64_t z = (s += 0x9E3779B97F4A7C15ULL);
        z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ULL;
        z = (z ^ (z >> 27)) * 0x94D049BB133111EBULL;
        return z ^ (z >> 31);
    }
    double uniform() { return (double)(next() >> 11) * 0x1.0p-53; }       // [0, 1)
    uint32_t below(uint32_t n) { return (uint32_t)(((unsigned __int128)next() * n) >> 64); }
};

// Zipf rejection-inversion sampler (Hörmann & Derflinger 1996), ranks 1..n.
struct Zipf {
    double s, hx1, hn, sconst;
    uint32_t n;
    static double helper1(double x) { return std::fabs(x) > 1e-8 ? std::log1p(x) / x : 1 - x * (0.5 - x * (1.0 / 3.0 - 0.25 * x)); }
    static double helper2(double x) { return std::fabs(x) > 1e-8 ? std::expm1(x) / x : 1 + x * 0.5 * (1 + x * (1.0 / 3.0) * (1 + 0.25 * x)); }
    double h(double x) const { return std::exp(-s * std::log(x)); }
    double hint(double x) const { double lx = std::log(x); return helper2((1 - s) * lx) * lx; }
    double hinv(double x) const { double t = x * (1 - s); if (t < -1) t = -1; return std::exp(helper1(t) * x); }
    Zipf(uint32_t n_, double s_) : s(s_), n(n_) {
        hx1 = hint(1.5) - 1.0;
        hn = hint(n + 0.5);
        sconst = 2 - hinv(hint(2.5) - h(2));
    }
    uint32_t sample(SplitMix64 &r) const {
        for (;;) {
            double u = hn + r.uniform() * (hx1 - hn);
            double x = hinv(u);
            double kd = std::floor(x + 0.5);
            if (kd < 1) kd = 1; else if (kd > n) kd = n;
            if (kd - x <= sconst || u >= hint(kd + 0.5) - h(kd)) return (uint32_t)kd;
        }
    }
};

template <typename T> T *dup(const std::vector<T> &v) {
    T *p = (T *)std::malloc(std::max<size_t>(1, v.size()) * sizeof(T));
    if (p && !v.empty()) std::memcpy(p, v.data(), v.size() * sizeof(T));
    return p;
}

} // namespace

extern "C" int32_t accord_workload_generate(const accord_workload_cfg *cfg, accord_batch *out)
{
    if (!cfg || !out || cfg->keyspace < 1 || cfg->keys_per_txn > cfg->keyspace || cfg->node_mod == 0 ||
        (cfg->range_frac > 0 && cfg->keyspace < 2))
        return ACCORD_ERR_ARG;
    std::memset(out, 0, sizeof(*out));
    const uint32_t n = cfg->n, ks = cfg->keyspace;
    SplitMix64 rng(cfg->seed);
    std::vector<uint32_t> perm(ks);
    for (uint32_t i = 0; i < ks; ++i) perm[i] = i;
    for (uint32_t i = ks - 1; i > 0; --i) std::swap(perm[i], perm[rng.below(i + 1)]);
    const bool zipf = cfg->zipf_s > 0;
    Zipf z(ks, zipf ? cfg->zipf_s : 1.0);

    std::vector<uint64_t> msb(n), lsb(n);
    std::vector<int32_t> node(n);
    std::vector<uint32_t> key_off(n + 1), key_ord, rng_off(n + 1), rng_start, rng_end;
    key_ord.reserve((size_t)n * cfg->keys_per_txn);
    std::vector<uint32_t> tmp;
    std::vector<std::pair<uint32_t, uint32_t>> rs;
    const uint64_t epoch = 1;
    for (uint32_t i = 0; i < n; ++i) {
        const uint64_t hlc = 1000000ULL + i;
        const bool is_range = cfg->range_frac > 0 && rng.uniform() < cfg->range_frac;
        uint32_t kind;
        if (is_range) kind = rng.uniform() < 0.5 ? 1u : 0u;
        else kind = rng.uniform() < cfg->write_frac ? 1u : 0u;
        const uint32_t flags = (kind << 1) | (is_range ? 1u : 0u);
        msb[i] = (epoch << 15) | (hlc >> 48);
        lsb[i] = (hlc << 16) | flags;
        node[i] = (int32_t)(1 + (i % cfg->node_mod));
        key_off[i] = (uint32_t)key_ord.size();
        rng_off[i] = (uint32_t)rng_start.size();
        if (!is_range) {
            tmp.clear();
            while (tmp.size() < cfg->keys_per_txn) {
                uint32_t k = zipf ? perm[z.sample(rng) - 1] : rng.below(ks);
                if (std::find(tmp.begin(), tmp.end(), k) == tmp.end()) tmp.push_back(k);
            }
            std::sort(tmp.begin(), tmp.end());
            key_ord.insert(key_ord.end(), tmp.begin(), tmp.end());
        } else {
            const uint32_t nr = 1 + rng.below(std::max(1u, cfg->ranges_max));
            rs.clear();
            for (uint32_t r = 0; r < nr; ++r) {
                uint32_t len = 1 + rng.below(std::max(1u, std::min(cfg->range_len_max, ks - 1)));
                uint32_t s = rng.below(ks - len);       // (s, s+len] within [0, ks)
                rs.emplace_back(s, s + len);
            }
            std::sort(rs.begin(), rs.end());
            std::vector<std::pair<uint32_t, uint32_t>> merged;
            for (auto &r : rs) {
                if (!merged.empty() && merged.back().second > r.first)   // strictly overlapping
                    merged.back().second = std::max(merged.back().second, r.second);
                else merged.push_back(r);
            }
            for (auto &r : merged) { rng_start.push_back(r.first); rng_end.push_back(r.second); }
        }
    }
    key_off[n] = (uint32_t)key_ord.size();
    rng_off[n] = (uint32_t)rng_start.size();
    out->n = n;
    out->msb = dup(msb); out->lsb = dup(lsb); out->node = dup(node);
    out->key_off = dup(key_off); out->key_ord = dup(key_ord);
    out->rng_off = dup(rng_off); out->rng_start = dup(rng_start); out->rng_end = dup(rng_end);
    if (!out->msb || !out->lsb || !out->node || !out->key_off || !out->key_ord || !out->rng_off
        || !out->rng_start || !out->rng_end) {
        accord_workload_free(out);
        return ACCORD_ERR_OOM;
    }
    return ACCORD_OK;
}

extern "C" void accord_workload_free(accord_batch *b)
{
    if (!b) return;
    std::free((void *)b->msb); std::free((void *)b->lsb); std::free((void *)b->node);
    std::free((void *)b->key_off); std::free((void *)b->key_ord);
    std::free((void *)b->rng_off); std::free((void *)b->rng_start); std::free((void *)b->rng_end);
    std::memset(b, 0, sizeof(*b));
}
