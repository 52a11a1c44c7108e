// av1r_pipeline.cpp -- many independent streams on one GPU, in native threads (include/av1r.h,
// "multi-stream pipeline"; SURVEY.md §8e batching + §8f rank 4 parse || GPU).
//
// One producer thread per stream pulls the stream's frames in decode order from a source
// (in-memory batches, or IVF temporal units parsed by the host parser) and packs each
// (av1r_pack: validation, dependency schedule, pinned copy) into the stream's queue, up to
// `depth` frames ahead.  The calling thread is the launcher: each round it takes the head of
// every stream that has one and is not running a key frame alone (av1r_busy), and decodes
// them in shared launches (av1r_decode_packed_batch); a show-existing frame is applied on its
// stream in order (av1r_show_existing).  This is the reference's per-stream Decoder::decode
// loop (decoder/Av1Decoder.cpp:49-109) with reconstruction batched across streams, and with
// no interpreter anywhere on the path.
#include <stdio.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <mutex>
#include <new>
#include <string>
#include <thread>
#include <vector>

#include "av1p.h"
#include "av1r.h"

namespace {

using Clock = std::chrono::steady_clock;
double secs(Clock::duration d) { return std::chrono::duration<double>(d).count(); }

struct Entry {
    av1r_packed* p = nullptr;
    int kind = 0;  // 0 packed frame, 1 show existing, 2 end of stream, 3 error
    int show = 0, refresh = 0;
    int status = 0;
};

struct StreamQ {
    std::mutex m;
    std::condition_variable space;
    std::deque<Entry> q;
    double produce_s = 0, pack_s = 0;
    std::string err;
};

struct Run {
    std::vector<StreamQ> qs;
    std::atomic<bool> stop{false};
    std::mutex wm;  // launcher wake-up
    std::condition_variable ready;
    int depth = 3;
    explicit Run(int n) : qs(n) {}

    void push(int s, const Entry& e)
    {
        StreamQ& Q = qs[s];
        {
            std::unique_lock<std::mutex> l(Q.m);
            Q.space.wait(l, [&] { return (int)Q.q.size() < depth || stop.load(); });
            if (stop.load() && e.p) {
                av1r_packed_free(e.p);
                return;
            }
            Q.q.push_back(e);
        }
        std::lock_guard<std::mutex> l(wm);
        ready.notify_one();
    }
};

void producer(Run* R, int s, const av1r_stream_source* src, int64_t maxFrames)
{
    StreamQ& Q = R->qs[s];
    int64_t made = 0;
    Entry e;
    while (!R->stop.load() && (maxFrames <= 0 || made < maxFrames)) {
        const av1r_frame_batch* b = nullptr;
        const auto t0 = Clock::now();
        const int rc = src->next(src->user, s, &b);
        const auto t1 = Clock::now();
        Q.produce_s += secs(t1 - t0);
        if (rc == 1) break;
        if (rc < 0 || !b || !b->hdr) {
            e = Entry();
            e.kind = 3;
            e.status = rc < 0 ? rc : AV1R_E_INVALID;
            Q.err = "stream " + std::to_string(s) + ": source failed";
            R->push(s, e);
            return;
        }
        e = Entry();
        if (b->hdr->show_existing_frame) {
            e.kind = 1;
            e.show = b->hdr->frame_to_show;
            e.refresh = b->hdr->refresh_frame_flags;
        } else {
            const int pr = av1r_pack(b, &e.p);
            Q.pack_s += secs(Clock::now() - t1);
            if (pr) {
                e.kind = 3;
                e.status = pr;
                Q.err = "stream " + std::to_string(s) + ": av1r_pack: " + av1r_pack_last_error();
                R->push(s, e);
                return;
            }
        }
        R->push(s, e);
        made++;
    }
    e = Entry();
    e.kind = 2;
    R->push(s, e);
}

// ---- built-in sources ----
struct IvfStream {
    const uint8_t* data = nullptr;
    size_t size = 0, pos = 32;
    av1p_ctx* parser = nullptr;
    int have = 0, next = 0;  // frames of the last unit, the next one to hand out
};
struct IvfSource {
    std::vector<IvfStream> st;
};

int ivf_next(void* user, int s, const av1r_frame_batch** out)
{
    IvfStream& S = ((IvfSource*)user)->st[s];
    while (S.next >= S.have) {
        if (S.pos + 12 > S.size) return 1;
        const uint32_t sz = S.data[S.pos] | S.data[S.pos + 1] << 8 | S.data[S.pos + 2] << 16 | (uint32_t)S.data[S.pos + 3] << 24;
        S.pos += 12;
        if (S.pos + sz > S.size) return AV1R_E_INVALID;
        int n = 0;
        const int rc = av1p_decode_tu(S.parser, S.data + S.pos, sz, &n);
        S.pos += sz;
        if (rc) return rc;
        S.have = n;
        S.next = 0;
    }
    *out = av1p_frame(S.parser, S.next++);
    return 0;
}

}  // namespace

extern "C" {

int av1r_cycle_next(void* user, int stream, const av1r_frame_batch** batch)
{
    av1r_cycle* c = (av1r_cycle*)user;
    if (!c || !batch || stream < 0 || c->count[stream] <= 0) return AV1R_E_INVALID;
    *batch = c->batches[stream][c->pos[stream] % c->count[stream]];
    c->pos[stream]++;
    return 0;
}

int av1r_ivf_source_create(const uint8_t* const* files, const size_t* sizes, int n, av1r_stream_source* out)
{
    if (!files || !sizes || n <= 0 || !out) return AV1R_E_INVALID;
    IvfSource* S = new (std::nothrow) IvfSource;
    if (!S) return AV1R_E_NOMEM;
    S->st.resize(n);
    for (int i = 0; i < n; i++) {
        IvfStream& t = S->st[i];
        t.data = files[i];
        t.size = sizes[i];
        int rc = (t.size < 32 || memcmp(t.data, "DKIF", 4)) ? AV1R_E_INVALID : av1p_create(&t.parser);
        if (!rc) t.pos = t.data[6] | t.data[7] << 8;  // header length
        if (rc) {
            for (auto& u : S->st)
                if (u.parser) av1p_destroy(u.parser);
            delete S;
            return rc;
        }
    }
    out->next = ivf_next;
    out->user = S;
    return AV1R_OK;
}

void av1r_ivf_source_destroy(av1r_stream_source* src)
{
    if (!src || !src->user) return;
    IvfSource* S = (IvfSource*)src->user;
    for (auto& u : S->st)
        if (u.parser) av1p_destroy(u.parser);
    delete S;
    src->user = nullptr;
}

int av1r_pipeline_run(av1r_ctx* const* ctxs, int n, const av1r_stream_source* src, int64_t max_frames, int depth,
                      av1r_pipeline_stats* stats)
{
    if (!ctxs || n <= 0 || n > 32 || !src || !src->next) return AV1R_E_INVALID;
    Run R(n);
    R.depth = depth > 0 ? depth : 3;
    const auto t0 = Clock::now();
    std::vector<std::thread> th;
    th.reserve(n);
    for (int s = 0; s < n; s++) th.emplace_back(producer, &R, s, src, max_frames);
    std::vector<bool> done(n, false);
    int live = n, rc = AV1R_OK;
    uint64_t frames = 0, batches = 0;
    double wait_s = 0;
    std::vector<av1r_ctx*> bc;
    std::vector<av1r_packed*> bp;
    std::string err;
    while (live > 0 && rc == AV1R_OK) {
        bc.clear();
        bp.clear();
        for (int s = 0; s < n && rc == AV1R_OK; s++) {
            if (done[s] || av1r_busy(ctxs[s]) == 1) continue;
            StreamQ& Q = R.qs[s];
            // show-existing frames of this stream apply in order ahead of its next frame
            for (;;) {
                Entry e;
                {
                    std::lock_guard<std::mutex> l(Q.m);
                    if (Q.q.empty()) break;
                    e = Q.q.front();
                    Q.q.pop_front();
                }
                Q.space.notify_one();
                if (e.kind == 0) {
                    bc.push_back(ctxs[s]);
                    bp.push_back(e.p);
                    break;
                }
                if (e.kind == 1) {
                    if ((rc = av1r_show_existing(ctxs[s], e.show, e.refresh))) err = av1r_last_error(ctxs[s]);
                    frames++;
                    if (rc) break;
                    continue;
                }
                if (e.kind == 3) {
                    rc = e.status;
                    std::lock_guard<std::mutex> l(Q.m);
                    err = Q.err;
                }
                done[s] = true;
                live--;
                break;
            }
        }
        if (!bc.empty()) {
            const int r = av1r_decode_packed_batch(bc.data(), bp.data(), (int)bc.size());
            for (auto* p : bp) av1r_packed_free(p);
            if (r && rc == AV1R_OK) {
                rc = r;
                err = av1r_last_error(bc[0]);
            }
            frames += bc.size();
            batches++;
        } else if (live > 0 && rc == AV1R_OK) {
            // nothing ready: a producer's push wakes us; a key frame running alone does not,
            // hence the short bound
            const auto w0 = Clock::now();
            std::unique_lock<std::mutex> l(R.wm);
            R.ready.wait_for(l, std::chrono::microseconds(50));
            wait_s += secs(Clock::now() - w0);
        }
    }
    // stop and drain the producers (an error ends the run early)
    R.stop.store(true);
    for (auto& Q : R.qs) {
        std::lock_guard<std::mutex> l(Q.m);
        Q.space.notify_all();
    }
    for (auto& t : th) t.join();
    double produce_s = 0, pack_s = 0;
    for (auto& Q : R.qs) {
        for (auto& e : Q.q)
            if (e.p) av1r_packed_free(e.p);
        produce_s += Q.produce_s;
        pack_s += Q.pack_s;
    }
    for (int s = 0; s < n; s++) {
        const int r = av1r_synchronize(ctxs[s]);
        if (r && rc == AV1R_OK) {
            rc = r;
            err = av1r_last_error(ctxs[s]);
        }
    }
    if (stats) {
        stats->frames = frames;
        stats->batches = batches;
        stats->elapsed_s = secs(Clock::now() - t0);
        stats->produce_s = produce_s;
        stats->pack_s = pack_s;
        stats->wait_s = wait_s;
    }
    if (rc) fprintf(stderr, "av1r_pipeline_run: %s\n", err.c_str());
    return rc;
}

}  // extern "C"
