// ops.cpp — descriptor planning and kernel launches over device pointers.
#include <cstdlib>
#include <cstring>

#include "ops.hpp"

#include <algorithm>
#include <climits>
#include <deque>
#include <cstring>
#include <map>

#include "kernels.hpp"
#include "sha_plan.hpp"

namespace mxec {

int check_km(int k, int m) {
    if (k + m > 255)
        return set_error(MXEC_E_TOO_MANY_SHARDS_255,
                         "too many shards: " + std::to_string(k) + " data + " + std::to_string(m) +
                             " parity = " + std::to_string(k + m) +
                             " > 255 (GF(2^8) limit). Increase --chunk-size");
    int rc = rs_check(k, m);
    if (rc) return set_error(rc, std::string("Reed-Solomon init error: ") + mxec_strerror(rc));
    return MXEC_OK;
}

int encode_coef(Device& dev, int k, int m, uint32_t* off) {
    std::vector<uint8_t> key = {'E', uint8_t(k), uint8_t(m)};
    {
        std::lock_guard<std::mutex> g(dev.coef_mu);
        auto it = dev.coef_index.find(key);
        if (it != dev.coef_index.end()) {
            *off = it->second.off;
            coef_note_use(it->second.gen, it->second.seq);
            return MXEC_OK;
        }
    }
    auto mat = rs_matrix(k, m);
    if (!mat) return set_error(MXEC_E_SINGULAR_MATRIX, "encoding matrix construction failed");
    GfMatrix rows(m, k);
    for (int i = 0; i < m; ++i)
        for (int j = 0; j < k; ++j) rows.at(i, j) = mat->at(k + i, j);
    return coef_offset(dev, key, coef_tables(rows), off);
}

int decode_coef(Device& dev, const DecodePlan& plan, bool data_only, uint32_t* off) {
    std::vector<uint8_t> key = {'D', uint8_t(plan.k), uint8_t(plan.m), uint8_t(data_only)};
    for (int v : plan.valid) key.push_back(uint8_t(v));
    key.push_back(0xFF);
    for (int v : plan.missing) key.push_back(uint8_t(v));
    return coef_offset(dev, key, plan.table, off);
}

int decode_plan(Device& dev, int k, int m, const uint8_t* present, bool data_only,
                std::shared_ptr<const DecodePlan>* plan, uint32_t* off) {
    const int total = k + m;
    Device::PatternKey key;
    key.kmf = uint32_t(k) | uint32_t(m) << 8 | uint32_t(data_only) << 16;
    int np = 0;
    for (int i = 0; i < total; ++i) {
        const bool p = present[i] != 0;
        np += p;
        key.mask[size_t(i >> 6)] |= uint64_t(p) << (i & 63);
    }
    plan->reset();
    *off = 0;
    if (np < k) return MXEC_OK;
    {
        std::lock_guard<std::mutex> g(dev.coef_mu);
        auto it = dev.patterns.find(key);
        if (it != dev.patterns.end()) {
            *plan = std::static_pointer_cast<const DecodePlan>(it->second.plan);
            *off = it->second.off;
            if (!(*plan)->missing.empty()) coef_note_use(it->second.gen, it->second.seq);
            return MXEC_OK;
        }
    }
    auto p = decode_cache().get(k, m, present, data_only);
    if (!p) return set_error(MXEC_E_SINGULAR_MATRIX, "decode matrix inversion failed");
    uint32_t o = 0;
    CoefUse mine;  // the table's generation, then noted for the caller's batch too
    if (!p->missing.empty()) {
        CoefUse* outer = coef_use_swap(&mine);
        const int rc = decode_coef(dev, *p, data_only, &o);
        coef_use_swap(outer);
        MXEC_TRY(rc);
        coef_note_use(mine.lo, mine.seq);
    }
    {
        std::lock_guard<std::mutex> g(dev.coef_mu);
        // Only remember the offset while its generation is live (a recycle
        // may have come between the upload and here).
        const uint64_t gen = mine.any() ? mine.lo : dev.coef_gen;
        if (gen + 1 >= dev.coef_gen) dev.patterns.emplace(key, Device::PatternVal{p, o, gen, mine.seq});
    }
    *plan = p;
    *off = o;
    return MXEC_OK;
}

int run_rs(Device& dev, Slot& slot, hipStream_t s, uint64_t shard_size, int k, int r,
           const std::vector<RsObject>& objs, DescArena* arena, bool tune, uint32_t max_blocks) {
    if (objs.empty() || r == 0) return MXEC_OK;
    const size_t n = objs.size();
    if (affinity_on(dev)) {
        std::vector<const void*> ps;
        for (const RsObject& ob : objs) {
            for (int j = 0; j < k; ++j) ps.push_back(ob.in[j]);
            for (int i = 0; i < r; ++i) ps.push_back(ob.out[i]);
        }
        MXEC_TRY(affinity_check(dev, &slot, s, "run_rs", arena, ps.data(), ps.size()));
    }
    DescWriter w(slot, arena);
    const uint64_t tile = rs_tile_bytes(rs_default_variant(uint32_t(r)));
    const uint64_t tiles_per_obj = (shard_size + tile - 1) / tile;
    bool aligned = true;
    for (size_t o = 0; o < n && aligned; ++o) {
        for (int j = 0; j < k; ++j) aligned &= (reinterpret_cast<uintptr_t>(objs[o].in[j]) & 15) == 0;
        for (int i = 0; i < r; ++i) aligned &= (reinterpret_cast<uintptr_t>(objs[o].out[i]) & 15) == 0;
    }
    // Aligned launches handle length boundaries inside the fast kernel; an
    // unaligned pointer sends every tile to the byte-exact edge kernel.
    std::vector<uint64_t> edges;
    if (!aligned)
        for (size_t o = 0; o < n; ++o)
            for (uint64_t t = 0; t < tiles_per_obj; ++t) edges.push_back(uint64_t(o) << 32 | t);
    const size_t o_in = w.add(sizeof(void*) * n * k);
    const size_t o_out = w.add(sizeof(void*) * n * r);
    const size_t o_inlen = w.add(8 * n * k);
    const size_t o_outlen = w.add(8 * n * r);
    const size_t o_coef = w.add(4 * n);
    const size_t o_edge = w.add(8 * edges.size());
    char* hb = w.data();
    auto** ip = reinterpret_cast<const uint8_t**>(hb + o_in);
    auto** op = reinterpret_cast<uint8_t**>(hb + o_out);
    auto* il = reinterpret_cast<uint64_t*>(hb + o_inlen);
    auto* ol = reinterpret_cast<uint64_t*>(hb + o_outlen);
    auto* co = reinterpret_cast<uint32_t*>(hb + o_coef);
    for (size_t o = 0; o < n; ++o) {
        const RsObject& ob = objs[o];
        for (int j = 0; j < k; ++j) {
            ip[o * k + j] = ob.in[j];
            il[o * k + j] = std::min<uint64_t>(ob.in_len[j], shard_size);
        }
        for (int i = 0; i < r; ++i) {
            op[o * r + i] = ob.out[i];
            ol[o * r + i] = std::min<uint64_t>(ob.out_len[i], shard_size);
        }
        co[o] = ob.coef_off;
    }
    if (!edges.empty()) std::memcpy(hb + o_edge, edges.data(), 8 * edges.size());
    char* db = nullptr;
    MXEC_TRY(w.commit(s, &db));
    RsArgs a{};
    a.in_ptrs = reinterpret_cast<const uint8_t* const*>(db + o_in);
    a.out_ptrs = reinterpret_cast<uint8_t* const*>(db + o_out);
    a.in_len = reinterpret_cast<const uint64_t*>(db + o_inlen);
    a.out_len = reinterpret_cast<const uint64_t*>(db + o_outlen);
    a.coef = static_cast<const uint32_t*>(dev.coef.p);
    a.coef_off = reinterpret_cast<const uint32_t*>(db + o_coef);
    a.edge_list = reinterpret_cast<const uint64_t*>(db + o_edge);
    a.n_edge = edges.size();
    a.edge_tile_bytes = tile;
    a.shard_size = shard_size;
    a.n_obj = uint32_t(n);
    a.k = uint32_t(k);
    a.r_total = uint32_t(r);
    a.aligned = aligned ? 1u : 0u;
    a.max_blocks = max_blocks ? max_blocks : dev.kn ? dev.kn->test_rs_grid : 0u;
    if (max_blocks) tune = false;
    // Large aligned single-launch batches take the grid tuner's pick.
    GridTuner::Trial trial;
    const double gb = double(n) * double(k + r) * double(shard_size) / 1e9;
    if (aligned && r <= 4 && tune) MXEC_TRY(rs_grid_pick(dev, k, r, shard_size, gb, &a.blocks_per_cu, &trial));
    hipError_t e = trial.a ? hipEventRecord(trial.a, s) : hipSuccess;
    for (int row0 = 0; row0 < r && e == hipSuccess; row0 += 8) {
        a.row0 = uint32_t(row0);
        a.r = uint32_t(std::min(8, r - row0));
        e = launch_rs_apply(a, dev.n_cus, s);
    }
    if (trial.a && e == hipSuccess) e = hipEventRecord(trial.b, s);
    if (trial.a) {
        if (e == hipSuccess) {
            rs_grid_record(dev, k, r, shard_size, trial);
        } else {  // the trial's events are ours to free on a failed launch
            (void)hipEventDestroy(trial.a);
            (void)hipEventDestroy(trial.b);
        }
    }
    MXEC_HIP(e);
    return w.finish(s);
}

namespace {
// Tuning pays only where a launch is long enough for the grid to matter
// and an event pair costs nothing next to it.
constexpr double kTuneMinGB = 1.0;

bool tuning_on(const Device& dev) {
    if (dev.kn && (!dev.kn->rs_tune || dev.kn->test_rs_grid)) return false;
#ifdef MXEC_LAB
    if (getenv("MXEC_RS_BPC")) return false;  // a lab override fixes the grid
#endif
    return true;
}

// The candidate with the best time per GB (ties: the lower index).
int tuner_best(const GridTuner::State& st) {
    int b = 0;
    for (int c = 1; c < GridTuner::kCands; ++c)
        if (st.best_ms_per_gb[c] < st.best_ms_per_gb[b]) b = c;
    return b;
}

// Reads every finished trial of a shape into its best times; decides once
// every candidate has two samples (launches 2-7 of the shape cycle through
// the three grids).
void tuner_poll(GridTuner::State& st) {
    for (size_t i = 0; i < st.pending.size();) {
        GridTuner::Trial& t = st.pending[i];
        if (hipEventQuery(t.b) != hipSuccess) {
            (void)hipGetLastError();
            ++i;
            continue;
        }
        float ms = 0;
        if (hipEventElapsedTime(&ms, t.a, t.b) == hipSuccess && t.gb > 0) {
            st.best_ms_per_gb[t.cand] = std::min(st.best_ms_per_gb[t.cand], double(ms) / t.gb);
            ++st.samples[t.cand];
        }
        (void)hipGetLastError();
        (void)hipEventDestroy(t.a);
        (void)hipEventDestroy(t.b);
        st.pending.erase(st.pending.begin() + long(i));
    }
    bool all = true;
    for (int c = 0; c < GridTuner::kCands; ++c) all = all && st.samples[c] >= 2;
    if (st.decided < 0 && all) st.decided = tuner_best(st);
}
}  // namespace

int rs_grid_pick(Device& dev, int k, int r, uint64_t shard_size, double gb, uint32_t* bpc,
                 GridTuner::Trial* trial) {
    *bpc = 0;
    if (!tuning_on(dev) || gb < kTuneMinGB) return MXEC_OK;
    std::lock_guard<std::mutex> g(dev.tuner.mu);
    const auto key = std::make_tuple(k, r, shard_size);
    // A server sees a handful of shapes; past 256 new ones keep the default.
    if (dev.tuner.states.size() >= 256 && !dev.tuner.states.count(key)) return MXEC_OK;
    GridTuner::State& st = dev.tuner.states[key];
    if (!st.cands[0]) {
        st.cands[0] = rs_default_variant(uint32_t(r)).blocks_per_cu;
        st.cands[1] = st.cands[0] / 2;  // r <= 2: 1024 / 512 / 256; r = 3, 4: 512 / 256 / 128
        st.cands[2] = st.cands[0] / 4;
    }
    tuner_poll(st);
    if (st.decided >= 0) {
        *bpc = uint32_t(st.cands[st.decided]);
        return MXEC_OK;
    }
    constexpr int kTrials = 2 * GridTuner::kCands;
    if (st.launches > kTrials) {
        // Launches 2-7 were the trials (two per grid) and some still run (a
        // caller that queues far ahead): the default grid until their events
        // complete -- never a host wait inside an enqueue-only call.
        if (st.pending.empty()) st.decided = tuner_best(st);
        *bpc = uint32_t(st.cands[st.decided >= 0 ? st.decided : 0]);
        return MXEC_OK;
    }
    const int l = st.launches++;
    if (l == 0) return MXEC_OK;  // first launch of a shape: cold, untimed
    trial->cand = (l - 1) % GridTuner::kCands;
    trial->gb = gb;
    MXEC_HIP(hipEventCreate(&trial->a));
    if (hipEventCreate(&trial->b) != hipSuccess) {
        (void)hipEventDestroy(trial->a);
        trial->a = nullptr;
        return set_error(MXEC_E_DEVICE, "hipEventCreate failed");
    }
    *bpc = uint32_t(st.cands[trial->cand]);
    return MXEC_OK;
}

void rs_grid_record(Device& dev, int k, int r, uint64_t shard_size, const GridTuner::Trial& trial) {
    std::lock_guard<std::mutex> g(dev.tuner.mu);
    dev.tuner.states[std::make_tuple(k, r, shard_size)].pending.push_back(trial);
}

int rs_grid_in_use(Device& dev, int k, int r, uint64_t shard_size) {
    const int def = rs_default_variant(uint32_t(r)).blocks_per_cu;
#ifdef MXEC_LAB
    if (const char* e = getenv("MXEC_RS_BPC")) {
        const int b = atoi(e);
        if (b > 0 && b <= 4096) return b;
    }
#endif
    std::lock_guard<std::mutex> g(dev.tuner.mu);
    auto it = dev.tuner.states.find(std::make_tuple(k, r, shard_size));
    if (it == dev.tuner.states.end()) return def;
    tuner_poll(it->second);
    return it->second.decided >= 0 ? it->second.cands[it->second.decided] : 0;
}

void rs_grid_release(Device& dev) {
    std::lock_guard<std::mutex> g(dev.tuner.mu);
    for (auto& kv : dev.tuner.states)
        for (auto& t : kv.second.pending) {
            (void)hipEventDestroy(t.a);
            (void)hipEventDestroy(t.b);
        }
    dev.tuner.states.clear();
}

int run_rs_mixed(Device& dev, Slot& slot, hipStream_t s, const std::map<int, std::vector<RsMixedObject>>& groups,
                 DescArena* arena, uint32_t cap) {
    // Which groups take the grouped kernel: every pointer 16-byte aligned,
    // r <= 8, index ranges that fit its 32-bit fields.  A call that is one
    // uniform group keeps the uniform kernel (no tile table).
    struct Plan {
        int r;
        const std::vector<RsMixedObject>* objs;
        uint64_t sum_k = 0, n_tiles = 0, tile = 0;
        size_t o_in = 0, o_out = 0, o_inlen = 0, o_outlen = 0, o_coef = 0, o_tiles = 0;
    };
    std::vector<Plan> grouped;
    std::vector<std::pair<int, const std::vector<RsMixedObject>*>> rest;
    // Per r: the aligned objects (grouped launch) and the others (per (k, S)
    // launches through run_rs, whose edge kernel takes unaligned pointers).
    std::deque<std::vector<RsMixedObject>> parts;
    for (const auto& g : groups) {
        const int r = g.first;
        if (g.second.empty() || r == 0) continue;
        auto& al = parts.emplace_back();
        auto& un = parts.emplace_back();
        for (const RsMixedObject& ob : g.second) {
            bool aligned = r <= 8;
            for (int j = 0; j < ob.k && aligned; ++j) aligned &= (reinterpret_cast<uintptr_t>(ob.o.in[j]) & 15) == 0;
            for (int i = 0; i < r && aligned; ++i) aligned &= (reinterpret_cast<uintptr_t>(ob.o.out[i]) & 15) == 0;
            (aligned ? al : un).push_back(ob);
        }
        if (!un.empty()) rest.emplace_back(r, &un);
        if (al.empty()) continue;
        bool uniform = true;
        Plan p{r, &al};
        p.tile = rs_tile_bytes(rs_group_variant(uint32_t(r)));
        for (const RsMixedObject& ob : al) {
            uniform &= ob.k == al[0].k && ob.shard_size == al[0].shard_size;
            p.sum_k += uint64_t(ob.k);
            p.n_tiles += (ob.shard_size + p.tile - 1) / p.tile;
        }
        const bool fits = al.size() <= UINT32_MAX && p.sum_k <= UINT32_MAX && p.n_tiles <= (uint64_t(1) << 32);
        if (fits && !(uniform && groups.size() == 1 && un.empty())) grouped.push_back(p);
        else rest.emplace_back(r, &al);
    }
    for (const auto& g : rest) {
        // One launch per (k, shard_size), in order of first appearance.
        std::map<std::pair<int, uint64_t>, std::vector<RsObject>> by;
        std::vector<std::pair<int, uint64_t>> order;
        for (const RsMixedObject& ob : *g.second) {
            auto key = std::make_pair(ob.k, ob.shard_size);
            auto& v = by[key];
            if (v.empty()) order.push_back(key);
            v.push_back(ob.o);
        }
        for (const auto& key : order)
            MXEC_TRY(run_rs(dev, slot, s, key.second, key.first, g.first, by[key], arena, true, cap));
    }
    if (grouped.empty()) return MXEC_OK;
    if (affinity_on(dev)) {
        std::vector<const void*> ps;
        for (const Plan& p : grouped)
            for (const RsMixedObject& ob : *p.objs) {
                for (int j = 0; j < ob.k; ++j) ps.push_back(ob.o.in[j]);
                for (int i = 0; i < p.r; ++i) ps.push_back(ob.o.out[i]);
            }
        MXEC_TRY(affinity_check(dev, &slot, s, "run_rs_mixed", arena, ps.data(), ps.size()));
    }
    // Two or more grouped launches of r <= kMultiR with the same tile: one
    // multi-r launch instead (rs_apply_multi; MXEC_RS_MULTI=0 keeps one
    // launch per r).
    const bool multi_on = !dev.kn || dev.kn->rs_multi;
    const uint32_t max_blocks = cap ? cap : dev.kn ? dev.kn->test_rs_grid : 0u;
    bool multi = multi_on && grouped.size() >= 2;
    uint64_t m_obj = 0, m_k = 0, m_tiles = 0;
    const uint64_t m_tile = rs_tile_bytes(rs_group_variant(kMultiR));
    for (const Plan& p : grouped) {
        multi = multi && p.r <= int(kMultiR) && p.tile == m_tile;
        m_obj += p.objs->size();
        m_k += p.sum_k;
        m_tiles += p.n_tiles;
    }
    multi = multi && m_obj <= UINT32_MAX / kMultiR && m_k <= UINT32_MAX && m_tiles <= (uint64_t(1) << 32);
    if (multi) {
        DescWriter w(slot, arena);
        const size_t o_in = w.add(sizeof(void*) * m_k);
        const size_t o_out = w.add(sizeof(void*) * m_obj * kMultiR);
        const size_t o_inlen = w.add(8 * m_k);
        const size_t o_outlen = w.add(8 * m_obj * kMultiR);  // zero: unused output entries
        const size_t o_coef = w.add(4 * m_obj);
        const size_t o_tiles = w.add(sizeof(RsTileRec) * m_tiles);
        char* hb = w.data();
        auto** ip = reinterpret_cast<const uint8_t**>(hb + o_in);
        auto** op = reinterpret_cast<uint8_t**>(hb + o_out);
        auto* il = reinterpret_cast<uint64_t*>(hb + o_inlen);
        auto* ol = reinterpret_cast<uint64_t*>(hb + o_outlen);
        auto* co = reinterpret_cast<uint32_t*>(hb + o_coef);
        auto* tr = reinterpret_cast<RsTileRec*>(hb + o_tiles);
        uint64_t o = 0, in0 = 0, t0 = 0;
        for (const Plan& p : grouped) {
            for (const RsMixedObject& ob : *p.objs) {
                for (int j = 0; j < ob.k; ++j) {
                    ip[in0 + j] = ob.o.in[j];
                    il[in0 + j] = std::min<uint64_t>(ob.o.in_len[j], ob.shard_size);
                }
                for (int i = 0; i < p.r; ++i) {
                    op[o * kMultiR + i] = ob.o.out[i];
                    ol[o * kMultiR + i] = std::min<uint64_t>(ob.o.out_len[i], ob.shard_size);
                }
                co[o] = ob.o.coef_off;
                const uint64_t nt = (ob.shard_size + m_tile - 1) / m_tile;
                const uint32_t kr = uint32_t(ob.k) | uint32_t(p.r) << 16;
                for (uint64_t t = 0; t < nt; ++t) tr[t0 + t] = RsTileRec{uint32_t(o), kr, uint32_t(in0), uint32_t(t)};
                in0 += uint64_t(ob.k);
                t0 += nt;
                ++o;
            }
        }
        char* db = nullptr;
        MXEC_TRY(w.commit(s, &db));
        RsArgs a{};
        a.in_ptrs = reinterpret_cast<const uint8_t* const*>(db + o_in);
        a.out_ptrs = reinterpret_cast<uint8_t* const*>(db + o_out);
        a.in_len = reinterpret_cast<const uint64_t*>(db + o_inlen);
        a.out_len = reinterpret_cast<const uint64_t*>(db + o_outlen);
        a.coef = static_cast<const uint32_t*>(dev.coef.p);
        a.coef_off = reinterpret_cast<const uint32_t*>(db + o_coef);
        a.n_obj = uint32_t(m_obj);
        a.r = a.r_total = kMultiR;
        a.row0 = 0;
        a.aligned = 1;
        a.multi = 1;
        a.tiles = reinterpret_cast<const RsTileRec*>(db + o_tiles);
        a.n_tiles = m_tiles;
        a.max_blocks = max_blocks;
        MXEC_HIP(launch_rs_apply(a, dev.n_cus, s));
        return w.finish(s);
    }
    // Every grouped launch's tables in one upload: one host-to-device copy
    // ahead of the launches instead of one between each pair of them (a
    // copy in the stream costs ~25-50 us of idle GPU at that point).
    DescWriter w(slot, arena);
    for (Plan& p : grouped) {
        const size_t n = p.objs->size();
        p.o_in = w.add(sizeof(void*) * p.sum_k);
        p.o_out = w.add(sizeof(void*) * n * p.r);
        p.o_inlen = w.add(8 * p.sum_k);
        p.o_outlen = w.add(8 * n * p.r);
        p.o_coef = w.add(4 * n);
        p.o_tiles = w.add(sizeof(RsTileRec) * p.n_tiles);
    }
    char* hb = w.data();
    for (const Plan& p : grouped) {
        const int r = p.r;
        auto** ip = reinterpret_cast<const uint8_t**>(hb + p.o_in);
        auto** op = reinterpret_cast<uint8_t**>(hb + p.o_out);
        auto* il = reinterpret_cast<uint64_t*>(hb + p.o_inlen);
        auto* ol = reinterpret_cast<uint64_t*>(hb + p.o_outlen);
        auto* co = reinterpret_cast<uint32_t*>(hb + p.o_coef);
        auto* tr = reinterpret_cast<RsTileRec*>(hb + p.o_tiles);
        uint64_t in0 = 0, t0 = 0;
        for (size_t o = 0; o < p.objs->size(); ++o) {
            const RsMixedObject& ob = (*p.objs)[o];
            for (int j = 0; j < ob.k; ++j) {
                ip[in0 + j] = ob.o.in[j];
                il[in0 + j] = std::min<uint64_t>(ob.o.in_len[j], ob.shard_size);
            }
            for (int i = 0; i < r; ++i) {
                op[o * r + i] = ob.o.out[i];
                ol[o * r + i] = std::min<uint64_t>(ob.o.out_len[i], ob.shard_size);
            }
            co[o] = ob.o.coef_off;
            const uint64_t nt = (ob.shard_size + p.tile - 1) / p.tile;
            for (uint64_t t = 0; t < nt; ++t)
                tr[t0 + t] = RsTileRec{uint32_t(o), uint32_t(ob.k), uint32_t(in0), uint32_t(t)};
            in0 += uint64_t(ob.k);
            t0 += nt;
        }
    }
    char* db = nullptr;
    MXEC_TRY(w.commit(s, &db));
    for (const Plan& p : grouped) {
        RsArgs a{};
        a.in_ptrs = reinterpret_cast<const uint8_t* const*>(db + p.o_in);
        a.out_ptrs = reinterpret_cast<uint8_t* const*>(db + p.o_out);
        a.in_len = reinterpret_cast<const uint64_t*>(db + p.o_inlen);
        a.out_len = reinterpret_cast<const uint64_t*>(db + p.o_outlen);
        a.coef = static_cast<const uint32_t*>(dev.coef.p);
        a.coef_off = reinterpret_cast<const uint32_t*>(db + p.o_coef);
        a.n_obj = uint32_t(p.objs->size());
        a.r = a.r_total = uint32_t(p.r);
        a.row0 = 0;
        a.aligned = 1;
        a.tiles = reinterpret_cast<const RsTileRec*>(db + p.o_tiles);
        a.n_tiles = p.n_tiles;
        a.max_blocks = max_blocks;
        MXEC_HIP(launch_rs_apply(a, dev.n_cus, s));
    }
    return w.finish(s);
}

int run_sha(Device& dev, Slot& slot, hipStream_t s, const std::vector<const uint8_t*>& ptrs,
            const std::vector<uint64_t>& lens, uint8_t* digests_dev, const uint8_t* expected_dev,
            uint8_t* ok_dev, const std::vector<uint64_t>* exp_idx, DescArena* arena, int form,
            const uint32_t** tmo_dev) {
    const size_t n = ptrs.size();
    if (tmo_dev) *tmo_dev = nullptr;
    if (!n) return MXEC_OK;
    if (affinity_on(dev)) {
        std::vector<const void*> ps(ptrs.begin(), ptrs.end());
        ps.push_back(digests_dev);
        ps.push_back(ok_dev);
        MXEC_TRY(affinity_check(dev, &slot, s, "run_sha", arena, ps.data(), ps.size()));
    }
    // The stream form: more 64-message groups than SIMDs, every message
    // 16-byte aligned, a caller that checks the timeout word, ring tables.
    // MXEC_SHA_FORM=stream forces it whenever it is allowed (tests); one,
    // split and lagpair pin the other forms the auto choice takes.
    const uint64_t groups = (n + 63) / 64, simds = uint64_t(dev.n_cus) * 4;
    const int env_form = dev.kn ? dev.kn->sha_form : 0;
    uint64_t longest = 0;
    for (uint64_t l : lens) longest = std::max(longest, l);
    const uint64_t seg_max = sha_stream_seg_max(longest, kShaSegBlocks);
    // The stream kernel's 32-bit item counter must not wrap (sha_plan.hpp).
    const bool items_fit = sha_stream_items_fit(n, seg_max, simds);
    bool stream = false;
    if (!items_fit) {
        // many messages plus one very long one: the split / one-wave forms
    } else if (tmo_dev && !arena && (form == 0 || form == 3) && n < (uint64_t(1) << 31)) {
        bool aligned = true;
        for (const uint8_t* p : ptrs) aligned = aligned && (reinterpret_cast<uintptr_t>(p) & 15) == 0;
        stream = aligned && (sha_stream_size(groups, simds) || form == 3 || env_form == 3);
    } else if (tmo_dev && !arena && env_form == 3 && n < (uint64_t(1) << 31)) {
        bool aligned = true;
        for (const uint8_t* p : ptrs) aligned = aligned && (reinterpret_cast<uintptr_t>(p) & 15) == 0;
        stream = aligned;
    }
    DescWriter w(slot, arena);
    const size_t o_p = w.add(sizeof(void*) * n);
    const size_t o_l = w.add(8 * n);
    const size_t o_e = exp_idx ? w.add(8 * n) : 0;
    // Zeroed by the upload: [0] item counter, [1] timeout code, [4 + g] progress.
    const size_t o_w = stream ? w.add(4 * (4 + groups)) : 0;
    char* hb = w.data();
    std::memcpy(hb + o_p, ptrs.data(), sizeof(void*) * n);
    std::memcpy(hb + o_l, lens.data(), 8 * n);
    if (exp_idx) std::memcpy(hb + o_e, exp_idx->data(), 8 * n);
    char* db = nullptr;
    MXEC_TRY(w.commit(s, &db));
    ShaArgs a{};
    a.ptrs = reinterpret_cast<const uint8_t* const*>(db + o_p);
    a.lens = reinterpret_cast<const uint64_t*>(db + o_l);
    a.digests = digests_dev;
    a.expected = expected_dev;
    a.exp_idx = exp_idx ? reinterpret_cast<const uint64_t*>(db + o_e) : nullptr;
    a.ok = ok_dev;
    a.n = uint32_t(n);
    a.n_cus = uint32_t(dev.n_cus);
    a.force = form == 3 && !stream ? 0 : form;
    if (a.force == 0 && (env_form == 1 || env_form == 2 || env_form == 6)) a.force = env_form;
    if (stream) {
        void* st = nullptr;
        MXEC_TRY(w.scratch(32 * n, &st));
        a.force = 3;
        a.work = reinterpret_cast<uint32_t*>(db + o_w);
        a.state = static_cast<uint32_t*>(st);
        // One persistent wave per SIMD: 1.54 TB/s hashed from 65 536 to
        // 98 304 x 1 MiB, the chip's INT32 issue ceiling for this mix; two
        // per SIMD measured slower (131 072 x 1 MiB: 132.5 vs 92.8 ms for the
        // one-wave form; profiles/r2_sha_stream_lab.txt).
        a.waves = uint32_t(simds);
        // Four waves per workgroup: the dispatcher spreads a workgroup's
        // waves over the CU's four SIMDs, while one-wave workgroups after an
        // HBM-heavy kernel landed two to a SIMD on ~100 SIMDs and none on as
        // many, and the segment chains through the doubled SIMDs ran the
        // launch at half speed (81 920 x 1 MiB after an 8 GiB write kernel:
        // 110 ms vs 56; tools/sha_stream_lab place / repeat,
        // profiles/r2_sha_stream_placement.txt).
        a.wg_waves = simds % 4 == 0 ? 4 : 1;
        a.seg_max = uint32_t(seg_max);
        *tmo_dev = a.work + 1;
    }
    MXEC_HIP(launch_sha256(a, s));
    return w.finish(s);
}

int run_sha_pieces(Device& dev, Slot& slot, hipStream_t s, const std::vector<const uint8_t*>& ptrs,
                   const std::vector<uint64_t>& lens, const std::vector<uint32_t>& slots,
                   const std::vector<uint64_t>& totals, uint32_t* state_dev, bool resume, uint8_t* digests_dev,
                   DescArena* arena, const uint8_t* expected_dev, uint8_t* ok_dev) {
    const size_t n = ptrs.size();
    if (!n) return MXEC_OK;
    if (lens.size() != n || slots.size() != n || totals.size() != n || !state_dev ||
        n > uint64_t(kShaLagMsgs) * uint64_t(dev.n_cus ? dev.n_cus : 256))
        return set_error(MXEC_E_INVALID_ARG, "sha pieces: table sizes or message count");
    for (size_t i = 0; i < n; ++i)
        if (totals[i] == kShaNotFinal ? lens[i] % 64 != 0 : totals[i] < lens[i])
            return set_error(MXEC_E_INVALID_ARG, "sha pieces: a mid-message piece must be whole 64-byte blocks");
    if (affinity_on(dev)) {
        std::vector<const void*> ps(ptrs.begin(), ptrs.end());
        ps.push_back(digests_dev);
        ps.push_back(state_dev);
        MXEC_TRY(affinity_check(dev, &slot, s, "run_sha_pieces", arena, ps.data(), ps.size()));
    }
    DescWriter w(slot, arena);
    const size_t o_p = w.add(sizeof(void*) * n);
    const size_t o_l = w.add(8 * n);
    const size_t o_t = w.add(8 * n);
    const size_t o_s = w.add(4 * n);
    char* hb = w.data();
    std::memcpy(hb + o_p, ptrs.data(), sizeof(void*) * n);
    std::memcpy(hb + o_l, lens.data(), 8 * n);
    std::memcpy(hb + o_t, totals.data(), 8 * n);
    std::memcpy(hb + o_s, slots.data(), 4 * n);
    char* db = nullptr;
    MXEC_TRY(w.commit(s, &db));
    ShaArgs a{};
    a.ptrs = reinterpret_cast<const uint8_t* const*>(db + o_p);
    a.lens = reinterpret_cast<const uint64_t*>(db + o_l);
    a.digests = digests_dev;
    a.expected = expected_dev;
    a.ok = ok_dev;
    a.n = uint32_t(n);
    a.n_cus = uint32_t(dev.n_cus);
    a.force = 6;
    a.piece.state = state_dev;
    a.piece.slot = reinterpret_cast<const uint32_t*>(db + o_s);
    a.piece.total = reinterpret_cast<const uint64_t*>(db + o_t);
    a.piece.resume = resume ? 1u : 0u;
    MXEC_HIP(launch_sha256(a, s));
    return w.finish(s);
}

}  // namespace mxec
