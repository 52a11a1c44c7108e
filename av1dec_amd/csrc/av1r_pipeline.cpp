// av1r_pipeline.cpp -- many independent streams on one GPU, in native threads (include/av1r.h,
// "multi-stream pipeline"; SURVEY.md §8e batching + §8f rank 4 parse || GPU).
//
// A pool of worker threads pulls every stream's frames in decode order from a source
// (in-memory batches, or IVF temporal units parsed by the host parser; one fetch per stream
// at a time) and packs them (av1r_pack: validation, dependency schedule, pinned copy), up to
// `depth` frames ahead per stream -- frames of one stream pack concurrently when the
// source's batches outlive the next fetch (`stable`).  The calling thread is the launcher: each round it takes the head of
// every stream that has one and is not running a key frame alone (av1r_busy), and decodes
// them in shared launches (av1r_decode_packed_batch); a show-existing frame is applied on its
// stream in order (av1r_show_existing).  This is the reference's per-stream Decoder::decode
// loop (decoder/Av1Decoder.cpp:49-109) with reconstruction batched across streams, and with
// no interpreter anywhere on the path.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <atomic>
#include <chrono>
#include <condition_variable>
#include <deque>
#include <algorithm>
#include <map>
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

// Per stream: frames are fetched from the source in order (one fetch at a time: seq numbers
// nextFetch), packed by any worker, and re-ordered by seq for the launcher (nextLaunch).
struct StreamQ {
    std::map<int64_t, Entry> ready;
    int64_t nextFetch = 0, nextLaunch = 0;
    bool pulling = false;  // a worker is inside src->next (or, unstable source, its pack)
    bool ended = false;    // the end / error entry has been queued
    double produce_s = 0, pack_s = 0;
    std::string err;
};

struct Run {
    std::vector<StreamQ> qs;
    const av1r_stream_source* src = nullptr;
    int64_t maxFrames = 0;
    int depth = 3;
    bool stable = false;  // src->stable != 0: the next fetch of a stream may overlap this pack
    std::atomic<bool> stop{false};
    std::mutex m;  // guards every StreamQ's bookkeeping (operations are tiny)
    std::condition_variable work, ready;
    int rr = 0;  // round-robin start of the workers' stream search
    explicit Run(int n) : qs(n) {}

    // a stream with room that nobody is fetching from, or -1
    int pick()
    {
        const int n = (int)qs.size();
        for (int k = 0; k < n; k++) {
            const int s = (rr + k) % n;
            StreamQ& Q = qs[s];
            if (Q.pulling || Q.ended || Q.nextFetch - Q.nextLaunch >= depth) continue;
            rr = (s + 1) % n;
            return s;
        }
        return -1;
    }
};

void worker(Run* R)
{
    std::unique_lock<std::mutex> l(R->m);
    while (!R->stop.load()) {
        const int s = R->pick();
        if (s < 0) {
            R->work.wait(l);
            continue;
        }
        StreamQ& Q = R->qs[s];
        const int64_t seq = Q.nextFetch++;
        Entry e;
        if (R->maxFrames > 0 && seq >= R->maxFrames) {  // this stream's share is done
            e.kind = 2;
            Q.ended = true;
            Q.ready[seq] = e;
            R->ready.notify_one();
            continue;
        }
        Q.pulling = true;
        l.unlock();
        const av1r_frame_batch* b = nullptr;
        const auto t0 = Clock::now();
        const int rc = R->src->next(R->src->user, s, &b);
        const auto t1 = Clock::now();
        double packS = 0;
        bool released = false;
        // (stable 2: the batch goes back to the source once packed)
        auto giveBack = [&]() {
            if (R->src->stable == 2 && R->src->release && rc == 0 && b) R->src->release(R->src->user, s, b);
        };
        if (rc == 0 && b && b->hdr && !b->hdr->show_existing_frame) {
            if (R->stable) {  // the batch outlives the next fetch: let another worker fetch
                l.lock();
                Q.pulling = false;
                R->work.notify_one();
                l.unlock();
                released = true;
            }
            const int pr = av1r_pack(b, &e.p);
            giveBack();
            packS = secs(Clock::now() - t1);
            if (pr) {
                e.kind = 3;
                e.status = pr;
                e.p = nullptr;
                l.lock();
                Q.err = "stream " + std::to_string(s) + ": av1r_pack: " + av1r_pack_last_error();
                l.unlock();
            }
        } else if (rc == 0 && b && b->hdr) {
            e.kind = 1;
            e.show = b->hdr->frame_to_show;
            e.refresh = b->hdr->refresh_frame_flags;
            giveBack();
        } else if (rc == 1) {
            e.kind = 2;
        } else {
            e.kind = 3;
            e.status = rc < 0 ? rc : AV1R_E_INVALID;
        }
        l.lock();
        if (!released) Q.pulling = false;
        if (e.kind == 3 && Q.err.empty()) Q.err = "stream " + std::to_string(s) + ": source failed";
        if (e.kind >= 2) Q.ended = true;
        Q.produce_s += secs(t1 - t0);
        Q.pack_s += packS;
        Q.ready[seq] = e;
        R->ready.notify_one();
        R->work.notify_one();
    }
}

// ---- built-in sources ----
// The IVF source keeps two generations of parsed frames (av1p_set_frame_generations): the
// frames of unit g stay valid while unit g + 1 is parsed, and before unit g + 2 is parsed
// (which recycles unit g's) every frame of unit g must be back (release): the next frame's
// parse runs while the pipeline packs this one (av1r_stream_source.stable = 2).
struct IvfStream {
    const uint8_t* data = nullptr;
    size_t size = 0, pos = 32;
    av1p_ctx* parser = nullptr;
    int have = 0, next = 0;  // frames of the last unit, the next one to hand out
    int64_t gen = 0;         // units parsed
    int out[2] = {0, 0};     // frames of unit gen - 1 / gen still held by the pipeline (by gen & 1)
    std::vector<std::pair<const av1r_frame_batch*, int64_t>> held;  // frames handed out, their unit
    std::mutex m;
    std::condition_variable back;
};
struct IvfSource {
    std::vector<IvfStream> st;
    explicit IvfSource(int n) : st(n) {}
};

int ivf_next(void* user, int s, const av1r_frame_batch** out)
{
    IvfStream& S = ((IvfSource*)user)->st[s];
    while (S.next >= S.have) {
        if (S.pos + 12 > S.size) return 1;
        const uint32_t sz = S.data[S.pos] | S.data[S.pos + 1] << 8 | S.data[S.pos + 2] << 16 | (uint32_t)S.data[S.pos + 3] << 24;
        S.pos += 12;
        if (S.pos + sz > S.size) return AV1R_E_INVALID;
        {  // parsing unit gen + 1 recycles unit gen - 1's frames: all of them back first
            std::unique_lock<std::mutex> l(S.m);
            S.back.wait(l, [&] { return S.out[(S.gen + 1) & 1] == 0; });
        }
        int n = 0;
        const int rc = av1p_decode_tu(S.parser, S.data + S.pos, sz, &n);
        S.pos += sz;
        if (rc) return rc;
        S.gen++;
        S.have = n;
        S.next = 0;
    }
    const av1r_frame_batch* b = av1p_frame(S.parser, S.next++);
    {
        std::lock_guard<std::mutex> l(S.m);
        S.out[S.gen & 1]++;
        S.held.push_back({b, S.gen});
    }
    *out = b;
    return 0;
}

void ivf_release(void* user, int s, const av1r_frame_batch* b)
{
    IvfStream& S = ((IvfSource*)user)->st[s];
    std::lock_guard<std::mutex> l(S.m);
    for (size_t i = 0; i < S.held.size(); i++)
        if (S.held[i].first == b) {
            S.out[S.held[i].second & 1]--;
            S.held.erase(S.held.begin() + i);
            S.back.notify_all();
            return;
        }
}

}  // namespace

extern "C" void av1r_pipe_prof_dump(double elapsed);  // av1r_host.cpp (AV1R_PIPE_PROF)

extern "C" {

int av1r_cycle_next(void* user, int stream, const av1r_frame_batch** batch)
{
    av1r_cycle* c = (av1r_cycle*)user;
    if (!c || !batch || stream < 0 || stream >= c->n_streams || c->count[stream] <= 0) return AV1R_E_INVALID;
    *batch = c->batches[stream][c->pos[stream] % c->count[stream]];
    c->pos[stream]++;
    return 0;
}

int av1r_ivf_source_create(const uint8_t* const* files, const size_t* sizes, int n, av1r_stream_source* out)
{
    if (!files || !sizes || n <= 0 || !out) return AV1R_E_INVALID;
    IvfSource* S = new (std::nothrow) IvfSource(n);
    if (!S) return AV1R_E_NOMEM;
    for (int i = 0; i < n; i++) {
        IvfStream& t = S->st[i];
        t.data = files[i];
        t.size = sizes[i];
        int rc = (t.size < 32 || memcmp(t.data, "DKIF", 4)) ? AV1R_E_INVALID : av1p_create(&t.parser);
        if (!rc) t.pos = t.data[6] | t.data[7] << 8;  // header length
        if (!rc) av1p_set_mode_info(t.parser, 0);      // av1r_pack rebuilds it on the device
        if (!rc) av1p_set_frame_generations(t.parser, 2);  // (IvfStream)
        if (rc) {
            for (auto& u : S->st)
                if (u.parser) av1p_destroy(u.parser);
            delete S;
            return rc;
        }
    }
    out->next = ivf_next;
    out->user = S;
    out->stable = 2;  // a unit's batches live until they are released (IvfStream)
    out->release = ivf_release;
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

}  // extern "C"

// A pipeline: the workers, the streams' queues and the launcher's per-stream positions.
// av1r_pipeline_run is open + one step + close; a pipeline kept open between steps keeps
// its workers packing `depth` frames ahead, so every step after the first runs in the
// steady state of a decoder that never stops (bench.py's warm-up and timed window).
struct av1r_pipeline {
    std::vector<av1r_ctx*> ctxs;
    Run R;
    std::vector<std::thread> th;
    std::vector<int64_t> launched;  // entries (frames, show-existing units) launched per stream
    std::vector<bool> ended;        // the stream's end (or error) entry was consumed
    int G = 1, g = 0;
    // frame delivery (av1r_pipeline_set_output): per stream the read-backs in flight, in order
    av1r_output_sink sink{};
    std::vector<std::deque<av1r_output_ticket*>> tick;
    // AV1R_PIPE_PROF=1: pipe_outputs' time (s) polling landed read-backs, blocked on the oldest
    // (in-flight cap), starting new ones, and draining at the step's end; tickets started
    double oprof[4] = {}, oissued = 0;
    explicit av1r_pipeline(int n) : R(n), launched(n, 0), ended(n, false), tick(n) {}
};

namespace {

int pipe_open(av1r_ctx* const* ctxs, int n, const av1r_stream_source* src, int64_t maxFrames, int depth, int workers,
              av1r_pipeline** out)
{
    av1r_pipeline* P = new (std::nothrow) av1r_pipeline(n);
    if (!P) return AV1R_E_NOMEM;
    P->ctxs.assign(ctxs, ctxs + n);
    Run& R = P->R;
    R.src = src;
    R.maxFrames = maxFrames;
    R.stable = src->stable != 0;
    const int W = std::max(1, std::min(workers > 0 ? workers : n, 64));
    // default look-ahead: enough packed frames per stream to keep every worker busy twice
    // over, at least 8 (measured on the box: 4K x 2 streams 410-445 frames/s at depth 3,
    // 530-600 at 5, 680-685 at 8; 1080p x 8 streams 3 370-3 450 / 3 470 / 3 610-3 670)
    R.depth = depth > 0 ? depth : std::max(8, 2 * ((W + n - 1) / n));
    // AV1R_PIPE_GROUPS=g: the streams form g groups whose batches go to g different HIP
    // streams (each batch runs on its first member's stream), so one group's latency-bound
    // k_flow overlaps the other groups' kernels
    // (default: one group.  Round 4 measured two groups from 8 streams faster -- 6 580-6 620
    // against 6 500 frames/s -- so a group's filters overlapped the other's reconstruction;
    // with round 6's kernels one group, launching all 8 streams' frames together as the
    // device-only leg does, is faster: 7 191-7 412 against 6 996-7 125 frames/s, 4 runs each,
    // profiles/r06_ab_pipe_groups.txt)
    static const int groups = getenv("AV1R_PIPE_GROUPS") ? std::max(1, atoi(getenv("AV1R_PIPE_GROUPS"))) : 1;
    P->G = std::min(groups, n);
    P->th.reserve(W);
    for (int w = 0; w < W; w++) P->th.emplace_back(worker, &R);
    *out = P;
    return AV1R_OK;
}

// Frame delivery: hand every landed read-back to the sink (in order per stream), then start
// the read-back of every frame the contexts have queued since (finish: wait for all of them).
// Runs on the launching thread between launches, so the copies overlap the next batches.
int pipe_outputs(av1r_pipeline* P, bool finish, std::string& err)
{
    if (!P->sink.acquire) return AV1R_OK;
    int rc = AV1R_OK;
    const int n = (int)P->ctxs.size();
    for (int s = 0; s < n; s++) {
        av1r_ctx* c = P->ctxs[s];
        auto& T = P->tick[s];
        auto deliverFront = [&](bool block) {
            av1r_output_ticket* t = T.front();
            if (!block) {
                const int q = av1r_output_query(t);
                if (q == 0) return false;
            }
            const int st = av1r_output_wait(t);
            T.pop_front();
            P->sink.deliver(P->sink.user, s, st);
            if (st && rc == AV1R_OK) {
                rc = st;
                err = av1r_last_error(c);
            }
            return true;
        };
        auto a0 = Clock::now();
        auto lap = [&](int k) {
            const auto a1 = Clock::now();
            P->oprof[k] += secs(a1 - a0);
            a0 = a1;
        };
        while (!T.empty() && deliverFront(false)) {
        }
        // the read-backs of the later frames whose decode has finished start now too (each
        // query issues its ticket's copies once the frame is ready; the copies run in order
        // on the context's read-back stream), so one slow front does not hold them back
        for (size_t i = 1; i < T.size(); i++)
            if (av1r_output_start(T[i]) == 0) break;
        lap(0);
        while (rc == AV1R_OK && av1r_output_pending(c) > 0) {
            if ((int)T.size() >= AV1R_SINK_INFLIGHT) {
                lap(2);
                deliverFront(true);
                lap(1);
            }
            P->oissued++;
            int w = 0, h = 0;
            uint8_t* pl[3] = {};
            int st[3] = {};
            int r = av1r_get_output(c, nullptr, 0, nullptr, 0, nullptr, 0, &w, &h);  // size only
            if (!r && P->sink.acquire(P->sink.user, s, w, h, pl, st)) {
                r = AV1R_E_INVALID;
                err = "stream " + std::to_string(s) + ": the output sink gave no buffer";
            }
            av1r_output_ticket* t = nullptr;
            if (!r && (r = av1r_get_output_async(c, pl[0], st[0], pl[1], st[1], pl[2], st[2], &w, &h, &t)))
                err = av1r_last_error(c);
            if (r) {
                rc = r;
                break;
            }
            T.push_back(t);
        }
        lap(2);
        while (finish && !T.empty()) deliverFront(true);
        lap(3);
    }
    return rc;
}

// Launch `frames` more entries of every stream (0: to the end of every stream), then
// synchronize every context.
int pipe_step(av1r_pipeline* P, int64_t frames, av1r_pipeline_stats* stats)
{
    Run& R = P->R;
    const int n = (int)P->ctxs.size();
    av1r_ctx* const* ctxs = P->ctxs.data();
    const auto t0 = Clock::now();
    std::vector<int64_t> tgt(n);
    std::vector<bool> done(n, false);
    int live = 0, rc = AV1R_OK;
    for (int s = 0; s < n; s++) {
        tgt[s] = frames > 0 ? P->launched[s] + frames : INT64_MAX;
        done[s] = P->ended[s] || P->launched[s] >= tgt[s];
        live += !done[s];
    }
    double produce0 = 0, pack0 = 0;
    {
        std::lock_guard<std::mutex> l(R.m);
        for (auto& Q : R.qs) {
            produce0 += Q.produce_s;
            pack0 += Q.pack_s;
        }
    }
    uint64_t nframes = 0, batches = 0;
    double wait_s = 0, launch_s = 0, output_s = 0;
    std::vector<av1r_ctx*> bc;
    std::vector<av1r_packed*> bp;
    std::string err;
    auto outputs = [&](bool finish) {
        const auto o0 = Clock::now();
        const int r = pipe_outputs(P, finish, err);
        output_s += secs(Clock::now() - o0);
        return r;
    };
    // (with a sink, one group: the read-backs share the group leads' upload streams, and two
    // leads uploading left them seldom idle -- the delivery leg fell to 0.84-0.88x)
    const int G = P->sink.acquire && !getenv("AV1R_PIPE_GROUPS") ? 1 : P->G;
    if (P->g >= G) P->g = 0;
    static const double fillUs = getenv("AV1R_PIPE_WAIT_US") ? atof(getenv("AV1R_PIPE_WAIT_US")) : 300.0;
    while (live > 0 && rc == AV1R_OK) {
        bc.clear();
        bp.clear();
        const int g = P->g;
        // group g: the g-th contiguous share of the streams (round 4: streams g, g + G, ...,
        // whose leads' streams land on different hardware queues -- contexts create two
        // streams each, dealt round-robin over 4 queues -- measured 6 490-6 540 against
        // 6 560-6 670 frames/s)
        const int sBeg = g * n / G, sEnd = (g + 1) * n / G, sStep = 1;
        P->g = (g + 1) % G;
        // full batches: while a stream that could join (live, not running a key frame alone)
        // has nothing packed yet, wait for it up to AV1R_PIPE_WAIT_US (bigger launches keep
        // the GPU busier than a partial batch launched early)
        if (fillUs > 0) {
            const auto f0 = Clock::now();
            std::unique_lock<std::mutex> l(R.m);
            for (;;) {
                int missing = 0;
                for (int s = sBeg; s < sEnd; s += sStep)
                    if (!done[s] && R.qs[s].ready.find(R.qs[s].nextLaunch) == R.qs[s].ready.end() && av1r_busy(ctxs[s]) != 1)
                        missing++;
                if (!missing || secs(Clock::now() - f0) * 1e6 >= fillUs) break;
                R.ready.wait_for(l, std::chrono::microseconds(20));
            }
            wait_s += secs(Clock::now() - f0);
        }
        for (int s = sBeg; s < sEnd && rc == AV1R_OK; s += sStep) {
            if (done[s] || av1r_busy(ctxs[s]) == 1) continue;
            StreamQ& Q = R.qs[s];
            // show-existing frames of this stream apply in order ahead of its next frame
            while (!done[s]) {
                Entry e;
                {
                    std::lock_guard<std::mutex> l(R.m);
                    auto it = Q.ready.find(Q.nextLaunch);
                    if (it == Q.ready.end()) break;
                    e = it->second;
                    Q.ready.erase(it);
                    Q.nextLaunch++;
                    if (e.kind == 3) err = Q.err;
                    R.work.notify_one();  // room for this stream again
                }
                if (e.kind == 0) {
                    bc.push_back(ctxs[s]);
                    bp.push_back(e.p);
                    if (++P->launched[s] >= tgt[s]) {
                        done[s] = true;
                        live--;
                    }
                    break;
                }
                if (e.kind == 1) {
                    if ((rc = av1r_show_existing(ctxs[s], e.show, e.refresh))) err = av1r_last_error(ctxs[s]);
                    nframes++;
                    if (++P->launched[s] >= tgt[s]) {
                        done[s] = true;
                        live--;
                    }
                    if (rc) break;
                    continue;
                }
                if (e.kind == 3) rc = e.status;
                P->ended[s] = true;
                done[s] = true;
                live--;
            }
        }
        if (!bc.empty()) {
            const auto l0 = Clock::now();
            const int r = av1r_decode_packed_batch(bc.data(), bp.data(), (int)bc.size());
            launch_s += secs(Clock::now() - l0);
            for (auto* p : bp) av1r_packed_free(p);
            if (r && rc == AV1R_OK) {
                rc = r;
                err = av1r_last_error(bc[0]);
            }
            nframes += bc.size();
            batches++;
            if (rc == AV1R_OK) rc = outputs(false);
        } else if (live > 0 && rc == AV1R_OK && P->g == 0) {
            // nothing ready in any group: a worker's push wakes us; a key frame running alone does not,
            // hence the short bound
            const auto w0 = Clock::now();
            std::unique_lock<std::mutex> l(R.m);
            R.ready.wait_for(l, std::chrono::microseconds(50));
            wait_s += secs(Clock::now() - w0);
            l.unlock();
            if (rc == AV1R_OK) rc = outputs(false);
        }
    }
    {  // every frame of the step delivered before it returns
        const int r = outputs(true);
        if (r && rc == AV1R_OK) rc = r;
    }
    for (int s = 0; s < n; s++) {
        const int r = av1r_synchronize(ctxs[s]);
        if (r && rc == AV1R_OK) {
            rc = r;
            err = av1r_last_error(ctxs[s]);
        }
    }
    if (stats) {
        double produce_s = 0, pack_s = 0;
        {
            std::lock_guard<std::mutex> l(R.m);
            for (auto& Q : R.qs) {
                produce_s += Q.produce_s;
                pack_s += Q.pack_s;
            }
        }
        stats->frames = nframes;
        stats->batches = batches;
        stats->elapsed_s = secs(Clock::now() - t0);
        stats->produce_s = produce_s - produce0;
        stats->pack_s = pack_s - pack0;
        stats->wait_s = wait_s;
        stats->launch_s = launch_s;
        stats->output_s = output_s;
    }
    if (rc) fprintf(stderr, "av1r_pipeline: %s\n", err.c_str());
    static const bool prof = getenv("AV1R_PIPE_PROF") && atoi(getenv("AV1R_PIPE_PROF")) != 0;
    if (prof && P->sink.acquire) {
        fprintf(stderr, "av1r_pipeline outputs: %.0f started; poll %.1f ms, blocked %.1f ms, start %.1f ms, drain %.1f ms\n",
                P->oissued, 1e3 * P->oprof[0], 1e3 * P->oprof[1], 1e3 * P->oprof[2], 1e3 * P->oprof[3]);
        P->oissued = 0;
        for (double& v : P->oprof) v = 0;
    }
    av1r_pipe_prof_dump(secs(Clock::now() - t0));
    return rc;
}

void pipe_close(av1r_pipeline* P)
{
    Run& R = P->R;
    for (auto& T : P->tick)  // read-backs of a failed step: released, not delivered
        for (av1r_output_ticket* t : T) (void)av1r_output_wait(t);
    {  // stop and drain the workers
        std::lock_guard<std::mutex> l(R.m);
        R.stop.store(true);
        R.work.notify_all();
    }
    for (auto& t : P->th) t.join();
    for (auto& Q : R.qs)
        for (auto& kv : Q.ready)
            if (kv.second.p) av1r_packed_free(kv.second.p);
    delete P;
}

bool cycle_ok(const av1r_stream_source* src, int n, int64_t frames)
{
    // a cycling source never ends: it needs a frame budget, and one batch list per stream
    return src->next != av1r_cycle_next ||
           (frames > 0 && src->user && static_cast<const av1r_cycle*>(src->user)->n_streams >= n);
}

}  // namespace

extern "C" {

int av1r_pipeline_run(av1r_ctx* const* ctxs, int n, const av1r_stream_source* src, int64_t max_frames, int depth,
                      int workers, av1r_pipeline_stats* stats)
{
    if (!ctxs || n <= 0 || n > 32 || !src || !src->next) return AV1R_E_INVALID;
    if (!cycle_ok(src, n, max_frames)) return AV1R_E_INVALID;
    av1r_pipeline* P = nullptr;
    int rc = pipe_open(ctxs, n, src, max_frames, depth, workers, &P);
    if (rc) return rc;
    rc = pipe_step(P, max_frames, stats);
    pipe_close(P);
    return rc;
}

int av1r_pipeline_open(av1r_ctx* const* ctxs, int n, const av1r_stream_source* src, int depth, int workers,
                       av1r_pipeline** out)
{
    if (!ctxs || n <= 0 || n > 32 || !src || !src->next || !out) return AV1R_E_INVALID;
    for (int i = 0; i < n; i++)
        if (!ctxs[i]) return AV1R_E_INVALID;
    if (src->next == av1r_cycle_next && (!src->user || static_cast<const av1r_cycle*>(src->user)->n_streams < n))
        return AV1R_E_INVALID;
    return pipe_open(ctxs, n, src, 0, depth, workers, out);
}

int av1r_pipeline_step(av1r_pipeline* p, int64_t frames, av1r_pipeline_stats* stats)
{
    if (!p) return AV1R_E_INVALID;
    if (!cycle_ok(p->R.src, (int)p->ctxs.size(), frames)) return AV1R_E_INVALID;
    return pipe_step(p, frames, stats);
}

int av1r_pipeline_set_output(av1r_pipeline* p, const av1r_output_sink* sink)
{
    if (!p || (sink && (!sink->acquire || !sink->deliver))) return AV1R_E_INVALID;
    for (auto& T : p->tick)
        if (!T.empty()) return AV1R_E_INVALID;  // (never between steps: a step delivers everything)
    p->sink = sink ? *sink : av1r_output_sink{};
    return AV1R_OK;
}

int av1r_pipeline_launched(const av1r_pipeline* p, int64_t* counts, int n)
{
    if (!p || !counts || n != (int)p->ctxs.size()) return AV1R_E_INVALID;
    for (int s = 0; s < n; s++) counts[s] = p->launched[s];
    return AV1R_OK;
}

void av1r_pipeline_close(av1r_pipeline* p)
{
    if (p) pipe_close(p);
}

}  // extern "C"
