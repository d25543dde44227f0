// async.cpp — completion-handle forms of the blocking host entry points.
//
// MaxIO calls the storage path from tokio workers (main.rs:81; the chunk
// reader runs inside poll_read, chunk_reader.rs:244-249).  A blocking
// mxec_reconstruct of a 1 MiB-chunk object takes ~30 ms (the SHA-256 chain),
// so a tokio caller would park a blocking-pool thread per request.  The
// *_async forms return at once with a ticket; the work runs on the context's
// own worker threads (one per slot, so every slot can have a call in flight)
// and the ticket's eventfd becomes readable when it is done — register it
// with tokio's AsyncFd and await readiness, then mxec_ticket_wait (which no
// longer blocks) for the result.  Pointer arrays and strings are copied at
// submission; data buffers and out-parameters must stay valid until the
// ticket completes.
#include <sys/eventfd.h>
#include <cerrno>
#include <unistd.h>

#include <condition_variable>
#include <deque>
#include <functional>
#include <string>
#include <thread>
#include <vector>

#include "../../include/maxio_ec.h"
#include "ops.hpp"

struct mxec_ticket {
    std::mutex mu;
    std::condition_variable cv;
    bool done = false;
    int rc = MXEC_OK;
    std::string msg;
    int efd = -1;
};

namespace mxec {

struct AsyncPool {
    std::mutex mu;
    std::condition_variable cv;
    std::deque<std::function<void()>> q;
    std::vector<std::thread> th;
    bool stop = false;

    explicit AsyncPool(size_t n) {
        for (size_t i = 0; i < n; ++i) th.emplace_back([this] { loop(); });
    }
    // Drains the queue, then joins (mxec_close: every submitted call finishes).
    ~AsyncPool() {
        {
            std::lock_guard<std::mutex> g(mu);
            stop = true;
        }
        cv.notify_all();
        for (auto& t : th)
            if (t.joinable()) t.join();
    }
    void loop() {
        for (;;) {
            std::function<void()> f;
            {
                std::unique_lock<std::mutex> lk(mu);
                cv.wait(lk, [&] { return stop || !q.empty(); });
                if (q.empty()) return;
                f = std::move(q.front());
                q.pop_front();
            }
            f();
        }
    }
    void submit(std::function<void()> f) {
        {
            std::lock_guard<std::mutex> g(mu);
            q.push_back(std::move(f));
        }
        cv.notify_one();
    }
};

void async_shutdown(Ctx& c) {
    std::shared_ptr<void> p;
    {
        std::lock_guard<std::mutex> g(c.pool_mu);
        p.swap(c.pool);
    }
    p.reset();  // joins the workers after the queue drained
}

namespace {

AsyncPool* pool_of(Ctx& c) {
    std::lock_guard<std::mutex> g(c.pool_mu);
    if (!c.pool) {
        size_t n = 0;
        for (auto& d : c.devs) n += d->slots.size();
        n = std::max<size_t>(2, std::min<size_t>(n, 64));
        c.pool = std::shared_ptr<void>(new AsyncPool(n), [](void* p) { delete static_cast<AsyncPool*>(p); });
    }
    return static_cast<AsyncPool*>(c.pool.get());
}

// Everything under the ticket's lock, `done` last: mxec_ticket_free frees
// the ticket (and closes its eventfd) as soon as it sees `done`, so the
// eventfd write and the notify must not follow the unlock.
void complete(mxec_ticket* t, int rc) {
    std::lock_guard<std::mutex> g(t->mu);
    t->rc = rc;
    t->msg = rc ? std::string(last_error()) : std::string();
    if (t->efd >= 0) {
        const uint64_t one = 1;
        ssize_t w;
        do {
            w = ::write(t->efd, &one, sizeof one);
        } while (w < 0 && errno == EINTR);
    }
    t->done = true;
    t->cv.notify_all();
}

// Queue `op` (returns an mxec status) on ctx's workers; *out gets the ticket.
int submit(mxec_ctx* ctx, mxec_ticket** out, std::function<int()> op) {
    if (!ctx || !out) return set_error(MXEC_E_INVALID_ARG, "null argument");
    auto* t = new mxec_ticket();
    t->efd = ::eventfd(0, EFD_CLOEXEC | EFD_NONBLOCK);
    if (t->efd < 0) {
        delete t;
        return set_error(MXEC_E_OOM, "eventfd failed");
    }
    try {
        pool_of(ctx->c)->submit([t, op = std::move(op)] {
            int rc;
            try {
                rc = op();
            } catch (...) {
                rc = set_error(MXEC_E_OOM, "host allocation failed");
            }
            complete(t, rc);
        });
    } catch (...) {
        ::close(t->efd);
        delete t;
        return set_error(MXEC_E_OOM, "could not queue the call");
    }
    *out = t;
    return MXEC_OK;
}

template <class T>
std::vector<T> copy_n(const T* p, size_t n) {
    return p ? std::vector<T>(p, p + n) : std::vector<T>();
}

}  // namespace
}  // namespace mxec

using namespace mxec;

extern "C" {

int mxec_ticket_fd(const mxec_ticket* t) { return t ? t->efd : -1; }

int mxec_ticket_poll(mxec_ticket* t) {
    if (!t) return set_error(MXEC_E_INVALID_ARG, "null ticket");
    std::lock_guard<std::mutex> g(t->mu);
    return t->done ? 1 : 0;
}

int mxec_ticket_wait(mxec_ticket* t) {
    if (!t) return set_error(MXEC_E_INVALID_ARG, "null ticket");
    std::unique_lock<std::mutex> lk(t->mu);
    t->cv.wait(lk, [&] { return t->done; });
    if (t->rc) set_error(t->rc, t->msg);
    return t->rc;
}

const char* mxec_ticket_error(const mxec_ticket* t) { return t ? t->msg.c_str() : ""; }

void mxec_ticket_free(mxec_ticket* t) {
    if (!t) return;
    {
        std::unique_lock<std::mutex> lk(t->mu);
        t->cv.wait(lk, [&] { return t->done; });
    }
    if (t->efd >= 0) ::close(t->efd);
    delete t;
}

int mxec_sha256_batch_async(mxec_ctx* ctx, const uint8_t* const* bufs, const size_t* lens, size_t n,
                            uint8_t (*out)[32], mxec_ticket** ticket) {
    return guarded([&] {
        if (n && (!bufs || !lens || !out)) return set_error(MXEC_E_INVALID_ARG, "null argument");
        auto b = copy_n(bufs, n);
        auto l = copy_n(lens, n);
        return submit(ctx, ticket, [=] { return mxec_sha256_batch(ctx, b.data(), l.data(), n, out); });
    });
}

int mxec_encode_async(mxec_ctx* ctx, int k, int m, size_t shard_size, const uint8_t* const* data,
                      const size_t* data_len, uint8_t* const* parity, uint8_t (*sha256_out)[32],
                      mxec_ticket** ticket) {
    return guarded([&] {
        MXEC_TRY(check_km(k, m));  // the crate / k+m>255 guards answer at once, as the blocking call would
        auto d = copy_n(data, size_t(k));
        auto dl = copy_n(data_len, size_t(k));
        auto p = copy_n(parity, size_t(m));
        const bool has_dl = data_len != nullptr, has_d = data != nullptr, has_p = parity != nullptr;
        return submit(ctx, ticket, [=] {
            return mxec_encode(ctx, k, m, shard_size, has_d ? d.data() : nullptr, has_dl ? dl.data() : nullptr,
                               has_p ? p.data() : nullptr, sha256_out);
        });
    });
}

int mxec_reconstruct_async(mxec_ctx* ctx, int k, int m, size_t shard_size, uint8_t* const* shards,
                           const size_t* shard_len, const uint8_t (*expected_sha256)[32], uint8_t* present_inout,
                           uint32_t flags, int* n_present, mxec_ticket** ticket) {
    return guarded([&] {
        if (int rc = mxec_rs_check(k, m)) return set_error(rc, std::string("RS init error: ") + mxec_strerror(rc));
        const size_t total = size_t(k + m);
        auto s = copy_n(shards, total);
        auto sl = copy_n(shard_len, total);
        std::vector<uint8_t> exp;
        if (expected_sha256) exp.assign(&expected_sha256[0][0], &expected_sha256[0][0] + 32 * total);
        const bool has_s = shards != nullptr, has_sl = shard_len != nullptr;
        return submit(ctx, ticket, [=] {
            return mxec_reconstruct(ctx, k, m, shard_size, has_s ? s.data() : nullptr, has_sl ? sl.data() : nullptr,
                                    exp.empty() ? nullptr : reinterpret_cast<const uint8_t(*)[32]>(exp.data()),
                                    present_inout, flags, n_present);
        });
    });
}

int mxec_reconstruct_strided_device_async(mxec_ctx* ctx, int dev, void* stream, int k, int m, uint64_t shard_size,
                                          uint64_t n_obj, uint8_t* shards, uint64_t obj_stride, uint64_t shard_stride,
                                          const uint64_t* shard_len, uint8_t* present,
                                          const uint8_t* expected_sha_dev, uint32_t flags, int32_t* status_out,
                                          mxec_ticket** ticket) {
    return guarded([&] {
        if (int rc = mxec_rs_check(k, m)) return set_error(rc, std::string("RS init error: ") + mxec_strerror(rc));
        if (shard_size == 0) return set_error(MXEC_E_EMPTY_SHARD, mxec_strerror(MXEC_E_EMPTY_SHARD));
        if (n_obj && (!shards || !present)) return set_error(MXEC_E_INVALID_ARG, "null argument");
        auto sl = copy_n(shard_len, size_t(k + m));
        const bool has_sl = shard_len != nullptr;
        return submit(ctx, ticket, [=] {
            return mxec_reconstruct_strided_device(ctx, dev, stream, k, m, shard_size, n_obj, shards, obj_stride,
                                                   shard_stride, has_sl ? sl.data() : nullptr, present,
                                                   expected_sha_dev, flags, status_out);
        });
    });
}

int mxec_reconstruct_batch_device_async(mxec_ctx* ctx, int dev, void* stream, const mxec_object* objs,
                                        uint64_t n_obj, uint8_t* const* shards, const uint64_t* shard_len,
                                        uint8_t* present, const uint8_t* expected_sha_dev, uint32_t flags,
                                        int32_t* status_out, mxec_ticket** ticket) {
    return guarded([&] {
        if (n_obj && (!objs || !shards || !present)) return set_error(MXEC_E_INVALID_ARG, "null argument");
        uint64_t sum = 0;
        for (uint64_t o = 0; o < n_obj; ++o) {
            if (int rc = mxec_rs_check(objs[o].k, objs[o].m))
                return set_error(rc, std::string("RS init error: ") + mxec_strerror(rc));
            if (objs[o].shard_size == 0) return set_error(MXEC_E_EMPTY_SHARD, mxec_strerror(MXEC_E_EMPTY_SHARD));
            sum += uint64_t(objs[o].k + objs[o].m);
        }
        // The object list, pointer and length arrays are copied here; present,
        // status_out and the shards stay the caller's until completion.
        auto ob = copy_n(objs, size_t(n_obj));
        auto sp = copy_n(shards, size_t(sum));
        auto sl = copy_n(shard_len, size_t(sum));
        const bool has_sl = shard_len != nullptr;
        return submit(ctx, ticket, [=] {
            return mxec_reconstruct_batch_device(ctx, dev, stream, ob.data(), n_obj, sp.data(),
                                                 has_sl ? sl.data() : nullptr, present, expected_sha_dev, flags,
                                                 status_out);
        });
    });
}

int mxec_put_object_chunked_async(mxec_ctx* ctx, const char* ec_dir, uint64_t chunk_size, uint32_t parity_shards,
                                  const uint8_t* body, size_t len, mxec_ticket** ticket) {
    return guarded([&] {
        if (!ec_dir) return set_error(MXEC_E_INVALID_ARG, "null argument");
        std::string dir(ec_dir);
        return submit(ctx, ticket, [=] {
            return mxec_put_object_chunked(ctx, dir.c_str(), chunk_size, parity_shards, body, len);
        });
    });
}

int mxec_get_object_chunked_async(mxec_ctx* ctx, const char* ec_dir, uint64_t offset, uint64_t length,
                                  uint8_t* out, uint64_t out_cap, uint64_t* out_len, mxec_ticket** ticket) {
    return guarded([&] {
        if (!ec_dir) return set_error(MXEC_E_INVALID_ARG, "null argument");
        std::string dir(ec_dir);
        return submit(ctx, ticket, [=] {
            return mxec_get_object_chunked(ctx, dir.c_str(), offset, length, out, out_cap, out_len);
        });
    });
}

}  // extern "C"
