// pipeline.cpp — replay buffer + concurrent self-play / training pipeline
// (SURVEY.md §8f.2): learner_concurrent.rs:244-290 (SelfPlayWorker::self_play_loop),
// :87-163 (ModelTrainerWorker::train_loop), main.rs:137-235 (train_concurrent).
//
//  * replay ring (HeapRb of capacity batch_size * 100, main.rs:142): pushes
//    overwrite the oldest samples (push_iter_overwrite), the trainer pops
//    batches from the oldest end (pop_iter().take(batch_size)) once at least
//    a batch is buffered (Condvar wait_while, learner_concurrent.rs:94-98);
//  * self-play workers: while training, refresh the net from the published
//    weights, play a batch of games on the device (spai_selfplay_run), push a
//    random 30 % subsample of the positions (choose_multiple, :278);
//  * trainer: train_iters x batches_per_iter device train steps
//    (spai_learner_train_batch), then save {dir}/{iter}.safetensors and publish
//    the weights (:153-161), then clear in_training (:163).
// Deviations: the self-play nets really take the trainer's weights (the
// reference's VarStore::copy before Net::new is a no-op, quirk Q9), and the
// subsample is drawn from Philox streams keyed by (seed, worker, batch) instead
// of thread_rng.  Everything runs on host threads over one or more GPUs: each
// worker owns an engine on its device, the learner owns one on its own.
#include <algorithm>
#include <atomic>
#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "philox.h"
#include "spai_internal.h"

struct spai_replay {
    uint32_t capacity = 0;
    std::vector<float> states, policies, values;   // [capacity][126], [capacity][7], [capacity]
    uint64_t head = 0;                             // index of the oldest sample
    uint32_t size = 0;
    uint64_t pushed = 0, popped = 0, overwritten = 0;
    std::mutex mu;
    std::condition_variable cv;
};

namespace spai {

constexpr int kEnc = 126, kPol = 7;

int replay_create(uint32_t capacity, spai_replay **out) {
    SPAI_CHECK(capacity > 0, SPAI_ERR_INVALID, "replay capacity must be > 0");
    spai_replay *r = new spai_replay();
    r->capacity = capacity;
    r->states.resize((size_t)capacity * kEnc);
    r->policies.resize((size_t)capacity * kPol);
    r->values.resize(capacity);
    *out = r;
    return SPAI_OK;
}

void replay_destroy(spai_replay *r) { delete r; }

// push_iter_overwrite: append in order; when full, the oldest sample is dropped.
// `ev` (optional) is completed with the ring size and handed to the observer
// while the lock is held, so observers see pushes and pops in ring order.
int replay_push(spai_replay *r, uint32_t n, const float *s, const float *p, const float *v,
                const Observer *obs) {
    {
        std::lock_guard<std::mutex> lk(r->mu);
        for (uint32_t i = 0; i < n; ++i) {
            if (r->size == r->capacity) {
                r->head = (r->head + 1) % r->capacity;
                r->size -= 1;
                r->overwritten += 1;
            }
            const size_t slot = (size_t)((r->head + r->size) % r->capacity);
            memcpy(&r->states[slot * kEnc], s + (size_t)i * kEnc, kEnc * 4);
            memcpy(&r->policies[slot * kPol], p + (size_t)i * kPol, kPol * 4);
            r->values[slot] = v[i];
            r->size += 1;
        }
        r->pushed += n;
        if (obs && obs->fn) {
            spai_pipeline_event ev = obs->ev;
            ev.kind = SPAI_PIPE_PUSH;
            ev.n = n;
            ev.ring_size = r->size;
            ev.states = s;
            ev.policies = p;
            ev.values = v;
            obs->fn(obs->user, &ev);
        }
    }
    r->cv.notify_all();
    return SPAI_OK;
}

// pop_iter().take(n) from the oldest end; wait_ms < 0 blocks until n are buffered
// (or `stop` is set), 0 fails at once when fewer are there
int replay_pop(spai_replay *r, uint32_t n, float *s, float *p, float *v, int wait_ms,
               const std::atomic<bool> *stop = nullptr, const Observer *obs = nullptr) {
    std::unique_lock<std::mutex> lk(r->mu);
    SPAI_CHECK(n <= r->capacity, SPAI_ERR_INVALID, "pop of %u from a ring of %u", n, r->capacity);
    auto ready = [&] { return r->size >= n || (stop && stop->load()); };
    if (wait_ms < 0) r->cv.wait(lk, ready);
    else if (wait_ms > 0) r->cv.wait_for(lk, std::chrono::milliseconds(wait_ms), ready);
    SPAI_CHECK(r->size >= n, SPAI_ERR_INVALID, "replay holds %u samples, %u requested", r->size, n);
    for (uint32_t i = 0; i < n; ++i) {
        const size_t slot = (size_t)((r->head + i) % r->capacity);
        memcpy(s + (size_t)i * kEnc, &r->states[slot * kEnc], kEnc * 4);
        memcpy(p + (size_t)i * kPol, &r->policies[slot * kPol], kPol * 4);
        v[i] = r->values[slot];
    }
    r->head = (r->head + n) % r->capacity;
    r->size -= n;
    r->popped += n;
    if (obs && obs->fn) {
        spai_pipeline_event ev = obs->ev;
        ev.kind = SPAI_PIPE_POP;
        ev.n = n;
        ev.ring_size = r->size;
        ev.states = s;
        ev.policies = p;
        ev.values = v;
        obs->fn(obs->user, &ev);
    }
    return SPAI_OK;
}

int replay_pop_now(spai_replay *r, uint32_t n, float *s, float *p, float *v) { return replay_pop(r, n, s, p, v, 0); }

int replay_size(spai_replay *r, uint32_t *n) {
    std::lock_guard<std::mutex> lk(r->mu);
    *n = r->size;
    return SPAI_OK;
}

// k distinct indices of [0, n) (choose_multiple): partial Fisher-Yates on a
// Philox stream keyed by (seed, stream id, draw counter)
void choose_multiple(uint32_t n, uint32_t k, uint64_t seed, uint64_t stream, std::vector<uint32_t> &out) {
    std::vector<uint32_t> idx(n);
    for (uint32_t i = 0; i < n; ++i) idx[i] = i;
    k = std::min(k, n);
    for (uint32_t i = 0; i < k; ++i) {
        uint32_t c[4] = {i, (uint32_t)stream, (uint32_t)(stream >> 32), 0x5A11u}, o[4];
        const uint32_t key[2] = {(uint32_t)seed, (uint32_t)(seed >> 32)};
        philox4x32(c, key, o);
        const uint64_t r64 = ((uint64_t)o[0] << 32) | o[1];
        const uint32_t j = i + (uint32_t)(r64 % (uint64_t)(n - i));
        std::swap(idx[i], idx[j]);
    }
    out.assign(idx.begin(), idx.begin() + k);
}

namespace {

struct Published {   // the trainer's latest weights (varstore_rwlock)
    std::mutex mu;
    std::vector<float> params;
    uint64_t version = 0;
};

struct Collect {     // one self-play batch's samples (sink target)
    std::vector<float> s, p, v;
};

void collect_sink(void *user, uint32_t, uint32_t n, const float *enc, const float *pol, const float *val,
                  const int32_t *) {
    Collect *c = (Collect *)user;
    c->s.insert(c->s.end(), enc, enc + (size_t)n * kEnc);
    c->p.insert(c->p.end(), pol, pol + (size_t)n * kPol);
    c->v.insert(c->v.end(), val, val + n);
}

}  // namespace

int pipeline_run(const spai_pipeline_config *cfg, const float *init_params, size_t n_params, spai_pipeline_stats *st) {
    SPAI_CHECK(cfg->n_selfplay >= 1 && cfg->selfplay_devices, SPAI_ERR_INVALID, "need >= 1 self-play worker");
    SPAI_CHECK(cfg->batch_size >= 1 && cfg->replay_capacity >= cfg->batch_size, SPAI_ERR_INVALID,
               "replay capacity %u < batch size %u", cfg->replay_capacity, cfg->batch_size);
    SPAI_CHECK(n_params == net_num_params(SPAI_GAME_CONNECT4, cfg->blocks, 64), SPAI_ERR_INVALID,
               "expected %zu params, got %zu", net_num_params(SPAI_GAME_CONNECT4, cfg->blocks, 64), n_params);
    const auto t0 = std::chrono::steady_clock::now();
    spai_replay *ring = nullptr;
    SPAI_TRY(replay_create(cfg->replay_capacity, &ring));
    Published pub;
    pub.params.assign(init_params, init_params + n_params);
    std::atomic<bool> in_training{true};
    std::atomic<bool> aborted{false};   // a worker failed: the trainer stops waiting for samples
    std::atomic<int> worker_rc{SPAI_OK};
    std::atomic<uint64_t> games{0}, positions{0}, max_version_used{0};
    std::string worker_err;
    std::mutex err_mu;

    auto worker = [&](uint32_t w) {   // SelfPlayWorker::self_play_loop
        spai_config ec{};
        spai_config_default(SPAI_GAME_CONNECT4, &ec);
        ec.c = cfg->c;
        ec.temperature = cfg->temperature;
        ec.num_searches = cfg->num_searches;
        ec.max_trees = cfg->games_per_batch;
        ec.eval = SPAI_EVAL_NET;
        ec.seed = cfg->seed;
        spai_engine *e = nullptr;
        spai_net *net = nullptr;
        uint64_t have = UINT64_MAX;
        int rc = spai_engine_create(SPAI_GAME_CONNECT4, &ec, cfg->selfplay_devices[w], &e);
        std::vector<float> params;
        std::vector<uint32_t> pick;
        for (uint64_t batch = 0; rc == SPAI_OK && in_training.load(); ++batch) {
            uint64_t ver;
            {
                std::lock_guard<std::mutex> lk(pub.mu);
                ver = pub.version;
                if (ver != have) params = pub.params;
            }
            if (ver != have) {   // refresh the self-play net from the published weights
                if (net) spai_net_destroy(net);
                net = nullptr;
                rc = spai_net_create(e, cfg->blocks, 64, params.data(), params.size(), SPAI_DTYPE_BF16, &net);
                if (rc == SPAI_OK) rc = spai_engine_set_net(e, net);
                have = ver;
            }
            if (rc != SPAI_OK) break;
            uint64_t prev = max_version_used.load();
            while (ver > prev && !max_version_used.compare_exchange_weak(prev, ver)) {
            }
            Collect col;
            spai_selfplay_stats sst{};
            const uint64_t gid = ((uint64_t)w << 40) + batch * cfg->games_per_batch;
            rc = spai_selfplay_run(e, cfg->games_per_batch, gid, collect_sink, &col, &sst);
            if (rc != SPAI_OK) break;
            const uint32_t n = (uint32_t)col.v.size();
            const uint32_t k = (uint32_t)((float)n * cfg->sample_fraction);   // (len as f32 * 0.3) as usize
            choose_multiple(n, k, cfg->seed, ((uint64_t)w << 32) | (uint32_t)batch, pick);
            std::vector<float> s((size_t)k * kEnc), p((size_t)k * kPol), v(k);
            for (uint32_t i = 0; i < k; ++i) {
                memcpy(&s[(size_t)i * kEnc], &col.s[(size_t)pick[i] * kEnc], kEnc * 4);
                memcpy(&p[(size_t)i * kPol], &col.p[(size_t)pick[i] * kPol], kPol * 4);
                v[i] = col.v[pick[i]];
            }
            Observer ob{cfg->observer, cfg->observer_user, spai_pipeline_event{}};
            ob.ev.worker = w;
            ob.ev.batch = batch;
            ob.ev.version = ver;
            ob.ev.positions = n;
            replay_push(ring, k, s.data(), p.data(), v.data(), &ob);
            games += cfg->games_per_batch;
            positions += n;
        }
        if (rc != SPAI_OK) {
            std::lock_guard<std::mutex> lk(err_mu);
            worker_err = spai_last_error();
            worker_rc = rc;
            in_training = false;
            aborted = true;
            ring->cv.notify_all();
        }
        if (net) spai_net_destroy(net);
        if (e) spai_engine_destroy(e);
    };

    std::vector<std::thread> threads;
    for (uint32_t w = 0; w < cfg->n_selfplay; ++w) threads.emplace_back(worker, w);

    // ModelTrainerWorker::train_loop on this thread
    int rc = SPAI_OK;
    spai_engine *le = nullptr;
    spai_learner *L = nullptr;
    double batches = 0, last[3] = {0, 0, 0};
    {
        spai_config ec{};
        spai_config_default(SPAI_GAME_CONNECT4, &ec);
        ec.max_trees = 1;
        rc = spai_engine_create(SPAI_GAME_CONNECT4, &ec, cfg->learner_device, &le);
        if (rc == SPAI_OK) rc = spai_learner_create(le, cfg->blocks, 64, init_params, n_params, nullptr, &L);
    }
    const uint32_t B = cfg->batch_size;
    std::vector<float> bs((size_t)B * kEnc), bp((size_t)B * kPol), bv(B), params(n_params);
    for (uint32_t it = 0; rc == SPAI_OK && it < cfg->train_iters; ++it) {
        for (uint32_t k = 0; rc == SPAI_OK && k < cfg->batches_per_iter; ++k) {
            Observer ob{cfg->observer, cfg->observer_user, spai_pipeline_event{}};
            ob.ev.batch = (uint64_t)batches;
            {
                std::lock_guard<std::mutex> lk(pub.mu);
                ob.ev.version = pub.version;
            }
            rc = replay_pop(ring, B, bs.data(), bp.data(), bv.data(), -1, &aborted, &ob);
            if (rc != SPAI_OK) break;   // only when the workers failed
            float loss[3];
            rc = spai_learner_train_batch(L, B, bs.data(), bp.data(), bv.data(), loss);
            if (rc == SPAI_OK) {
                batches += 1;
                for (int i = 0; i < 3; ++i) last[i] = loss[i];
            }
        }
        if (rc != SPAI_OK) break;
        rc = spai_learner_params(L, params.data(), n_params);
        if (rc == SPAI_OK && cfg->checkpoint_dir) {   // {checkpoint_dir}/{i}.safetensors (learner_concurrent.rs:155)
            const std::string path = std::string(cfg->checkpoint_dir) + "/" + std::to_string(it) + ".safetensors";
            rc = spai_params_save_safetensors(SPAI_GAME_CONNECT4, cfg->blocks, 64, params.data(), n_params,
                                              path.c_str());
        }
        if (rc == SPAI_OK) {
            std::lock_guard<std::mutex> lk(pub.mu);
            pub.params = params;
            pub.version = it + 1;
        }
    }
    const std::string trainer_err = rc == SPAI_OK ? "" : spai_last_error();
    in_training = false;   // *in_training_rwlock.write() = false (learner_concurrent.rs:163)
    ring->cv.notify_all();
    for (auto &t : threads) t.join();
    if (L) spai_learner_destroy(L);
    if (le) spai_engine_destroy(le);
    if (st) {
        st->games = (double)games.load();
        st->positions = (double)positions.load();
        st->samples_pushed = (double)ring->pushed;
        st->samples_overwritten = (double)ring->overwritten;
        st->batches_trained = batches;
        for (int i = 0; i < 3; ++i) st->last_loss[i] = last[i];
        st->weight_version_published = (double)pub.version;
        st->weight_version_used_max = (double)max_version_used.load();
        st->seconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    }
    replay_destroy(ring);
    if (worker_rc != SPAI_OK) {   // a failed worker also stops the trainer: report the cause
        set_error("self-play worker failed: %s", worker_err.c_str());
        return worker_rc;
    }
    if (rc != SPAI_OK) set_error("%s", trainer_err.c_str());
    return rc;
}

}  // namespace spai
