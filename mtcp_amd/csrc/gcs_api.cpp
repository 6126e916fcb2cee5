// gcs_api.cpp -- the extern "C" ABI of libmtcp_gpucsum.so (include/mtcp_gpucsum.h).
//
// Host-side runtime: per-thread contexts bound to one HIP device and one
// non-blocking stream (mTCP's one-context-per-core model, core.c:1153-1245),
// pinned staging for host batches with two slots so that the CPU gather of
// chunk k+1 overlaps the H2D/kernel/D2H of chunk k, and only verdicts (1 B per
// frame) or check fields (4 B per frame) come back over PCIe.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <atomic>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <memory>
#include <mutex>
#include <new>
#include <system_error>
#include <thread>
#include <vector>

#include <emmintrin.h>
#include <sched.h>
#include <sys/prctl.h>
#include <time.h>

#include "gcs_internal.h"

namespace {

thread_local char g_hip_err[256] = "";

int hip_fail(hipError_t e, const char* what)
{
    std::snprintf(g_hip_err, sizeof g_hip_err, "%s: %s (%d)", what, hipGetErrorString(e), (int)e);
    if (e == hipErrorOutOfMemory)
        return GCS_ENOMEM;
    if (e == hipErrorNoDevice || e == hipErrorInvalidDevice)
        return GCS_ENODEV;
    return GCS_EHIP;
}

// No C++ exception may cross the C ABI (mtcp_gpucsum.h: "no C++ exceptions
// cross the ABI"): every extern "C" entry point is a function-try-block whose
// handler maps the in-flight exception to a status code.
int exception_code() noexcept
{
    try {
        throw;
    } catch (const std::bad_alloc&) {
        std::snprintf(g_hip_err, sizeof g_hip_err, "C++ exception: std::bad_alloc");
        return GCS_ENOMEM;
    } catch (const std::exception& e) {
        std::snprintf(g_hip_err, sizeof g_hip_err, "C++ exception: %s", e.what());
        return GCS_EHIP;
    } catch (...) {
        std::snprintf(g_hip_err, sizeof g_hip_err, "C++ exception (unknown type)");
        return GCS_EHIP;
    }
}

#define GCS_CATCH \
    catch (...) { return exception_code(); }

// Test-only fault injection (tests/test_gpu_host.py): GCS_FAULT_INJECT names
// the failure to simulate.  Read per use; unset in production.
bool fault(const char* what)
{
    const char* e = std::getenv("GCS_FAULT_INJECT");
    return e && std::strcmp(e, what) == 0;
}

#define HIP_TRY(call)                                     \
    do {                                                  \
        hipError_t e_ = (call);                           \
        if (e_ != hipSuccess) return hip_fail(e_, #call); \
    } while (0)

constexpr int kSlots = 2;
constexpr uint64_t kSlotAlign = 64;   // pslib packing, io_engine/lib/pslib.c:146
// Host batches staged in at most this many bytes run in direct mode (the
// kernel reads pinned staging over PCIe; run_host_batch).  Per-call latency,
// DMA copies vs direct (tools/burst_lat.py): 64 x 1500 B verify
// 42 -> 21 us, 256 x 1500 B 87 -> 29 us, 1024 x 1500 B 136 -> 96 us.  The env
// variable GCS_DIRECT_MAX_BYTES overrides it (0 disables direct mode).
constexpr uint64_t kDirectMaxBytes = 2u << 20;

struct Slot {
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    uint8_t* h_frames = nullptr;   // pinned
    uint8_t* d_frames = nullptr;
    uint64_t* h_off = nullptr;
    uint64_t* d_off = nullptr;
    uint16_t* h_len = nullptr;
    uint16_t* d_len = nullptr;
    uint8_t* h_code = nullptr;
    uint8_t* d_code = nullptr;
    uint32_t* h_csum = nullptr;
    uint32_t* d_csum = nullptr;
    uint32_t* h_hash = nullptr;    // RSS outputs (gcs_classify*)
    uint32_t* d_hash = nullptr;
    uint16_t* h_queue = nullptr;
    uint16_t* d_queue = nullptr;
    uint64_t* h_rec = nullptr;     // direct mode: 8 B records (k_desc_rec), pinned
    // device views of the pinned buffers (direct mode: the kernel reads the
    // staged frames and writes its results over PCIe, no DMA copies)
    uint8_t* m_frames = nullptr;
    uint64_t* m_off = nullptr;
    uint16_t* m_len = nullptr;
    uint8_t* m_code = nullptr;
    uint32_t* m_csum = nullptr;
    uint32_t* m_hash = nullptr;
    uint16_t* m_queue = nullptr;
    uint64_t* m_rec = nullptr;
    // GCS_DIRECT_STAGE=device: a direct-mode batch is gathered into this
    // fine-grained device memory (host writes over the BAR, posted) instead
    // of the pinned staging, so the kernel reads its frames from HBM rather
    // than over PCIe; allocated on first use (ctx->direct_max bytes)
    uint8_t* v_frames = nullptr;
    // bookkeeping of the chunk in flight
    bool busy = false;
    bool served = false;           // results already complete (burst server)
    bool rec = false;              // results came as records (h_rec): unpack first
    uint32_t first = 0, count = 0;
};

}  // namespace

namespace {

// A few host threads that copy frames into pinned staging in parallel (one
// memcpy stream cannot feed PCIe Gen5).  Parts are handed out by an atomic
// counter; the calling thread works too and returns when every part is done.
class GatherPool {
  public:
    ~GatherPool()
    {
        {
            std::lock_guard<std::mutex> lk(m_);
            stop_ = true;
        }
        cv_.notify_all();
        for (auto& t : workers_)
            t.join();
    }

    void run(uint32_t total, uint32_t parts, const std::function<void(uint32_t, uint32_t)>& fn)
    {
        if (!started_)
            start();
        {
            std::lock_guard<std::mutex> lk(m_);
            job_ = &fn;
            total_ = total;
            parts_ = parts;
            done_ = 0;
            next_.store(0);
            gen_++;
        }
        cv_.notify_all();
        work();
        std::unique_lock<std::mutex> lk(m_);
        cv_done_.wait(lk, [&] { return done_ == parts_; });
        job_ = nullptr;
    }

    static int threads()
    {
        const char* e = std::getenv("GCS_GATHER_THREADS");
        int n = e ? std::atoi(e) : 8;
        return n < 1 ? 1 : (n > 64 ? 64 : n);
    }

  private:
    // Spawn the helpers.  A thread that cannot be created is not an error:
    // the calling thread always works through every part itself (work()), so
    // fewer helpers only means less parallel copying.
    void start()
    {
        started_ = true;
        for (int i = 1; i < threads(); i++) {
            try {
                if (fault("gather_thread"))
                    throw std::system_error(std::make_error_code(std::errc::resource_unavailable_try_again));
                workers_.emplace_back([this] { loop(); });
            } catch (const std::system_error&) {
                break;
            }
        }
    }

    void loop()
    {
        uint64_t seen = 0;
        for (;;) {
            {
                std::unique_lock<std::mutex> lk(m_);
                cv_.wait(lk, [&] { return stop_ || gen_ != seen; });
                if (stop_)
                    return;
                seen = gen_;
            }
            work();
        }
    }

    void work()
    {
        for (;;) {
            const uint32_t p = next_.fetch_add(1);
            const std::function<void(uint32_t, uint32_t)>* job;
            uint32_t parts, total;
            {
                std::lock_guard<std::mutex> lk(m_);
                job = job_;
                parts = parts_;
                total = total_;
            }
            if (!job || p >= parts)
                return;
            (*job)((uint32_t)((uint64_t)total * p / parts),
                   (uint32_t)((uint64_t)total * (p + 1) / parts));
            std::lock_guard<std::mutex> lk(m_);
            if (++done_ == parts_)
                cv_done_.notify_all();
        }
    }

    std::vector<std::thread> workers_;
    std::mutex m_;
    std::condition_variable cv_, cv_done_;
    const std::function<void(uint32_t, uint32_t)>* job_ = nullptr;
    uint32_t total_ = 0, parts_ = 0, done_ = 0;
    std::atomic<uint32_t> next_{0};
    uint64_t gen_ = 0;
    bool stop_ = false;
    bool started_ = false;
};

}  // namespace

namespace {

// Host side of the burst server (gcs_kernels.hip k_burst_server).  One
// ServerHub per device and process owns the resident grid, its stream and the
// mailbox; each context with the server on owns one of its request rings
// (BurstServer).  Small host batches in direct mode are posted to the ring
// instead of one kernel launch + event wait each.  The grid lives at most
// life_us and leaves after idle_us without work; a ring whose request finds
// the grid gone (or going) starts a fresh one, which resumes every ring where
// each block left it (HubPub::prog), so every request completes, none is
// served twice, and the grid never outlives its bounds.  Callers hold the
// device current (DeviceGuard).
class ServerHub {
  public:
    static ServerHub* get(int device)
    {
        if (device < 0 || device >= kMaxDevices)
            return nullptr;
        std::lock_guard<std::mutex> lk(registry_mu());
        ServerHub** hubs = registry();
        if (!hubs[device]) {
            // process lifetime: never freed (a static destructor would run
            // after the HIP runtime may have gone)
            std::unique_ptr<ServerHub> h(new ServerHub());
            if (h->init(device) != GCS_OK)
                return nullptr;
            hubs[device] = h.release();
        }
        return hubs[device];
    }

    // The device's hub if one was made (gcs_device_check), else nullptr.
    static ServerHub* peek(int device)
    {
        if (device < 0 || device >= kMaxDevices)
            return nullptr;
        std::lock_guard<std::mutex> lk(registry_mu());
        return registry()[device];
    }

    // gcs_device_check: with no ring joined, no grid may be resident and the
    // hub's stream must be idle (a grid outliving its contexts would serve
    // request lines whose frames were freed).
    int check_idle()
    {
        std::lock_guard<std::mutex> lk(mu_);
        if (mask_ != 0)
            return GCS_OK;
        if (launched_.load(std::memory_order_relaxed)) {
            std::snprintf(g_hip_err, sizeof g_hip_err,
                          "burst server: a grid is resident with no ring joined");
            return GCS_EHIP;
        }
        const hipError_t e = hipStreamQuery(stream_);
        if (e == hipErrorNotReady) {
            std::snprintf(g_hip_err, sizeof g_hip_err,
                          "burst server: the hub stream is busy with no ring joined");
            return GCS_EHIP;
        }
        return e == hipSuccess ? GCS_OK : hip_fail(e, "burst server stream");
    }

    // A context joins: ring index in *r, or GCS_ERANGE when kHubRings
    // contexts of this process already use the device's grid.  The grid
    // leaves first (it serves the rings of its launch only).
    int join(uint32_t start, int* r)
    {
        std::lock_guard<std::mutex> lk(mu_);
        int k = 0;
        while (k < gcs::kHubRings && ((mask_ >> k) & 1u))
            k++;
        if (k == gcs::kHubRings)
            return GCS_ERANGE;
        int rc = stop_locked();
        if (rc) return rc;
        read_knobs();
        std::memset(&mb_->ring[k], 0, sizeof(gcs::ServerMailbox));
        std::memset(&rq_->req[k], 0, sizeof rq_->req[k]);
        std::memset(&rq_->prof[k], 0, sizeof rq_->prof[k]);
        // every slot reads as holding `start` (done): a slot left at 0 would
        // read as NEWER than the next request near the 32-bit wrap, and be
        // skipped as done (line A whole: its tag half carries start too)
        for (auto& sl : rq_->req[k]) {
            sl.a.seq = start;
            sl.a.n = gcs::server_tag(start) << 16;
        }
        if (dev_mailbox_)
            _mm_sfence();                 // write-combined over the BAR
        // ... and every block's ack reads as `start` (nothing served yet): an
        // ack left at 0 would read as NEWER than a request >= 2^31 past it,
        // and complete an in-place request before its release fence
        // (test-only, GCS_FAULT_INJECT=ack_skew with GCS_SERVER_ACK_SKEW: join
        // with acks that stale, as after 2^31 requests that wrote no frame;
        // the grid must refresh them)
        const char* sk = fault("ack_skew") ? std::getenv("GCS_SERVER_ACK_SKEW") : nullptr;
        const uint32_t skew = sk ? (uint32_t)std::strtoul(sk, nullptr, 0) : 0u;
        for (auto& a : mb_->ring[k].ack)
            a.v = start + skew;
        // the ring starts at `start` on the device too: nothing claimed yet
        uint32_t prog[gcs::kServerBlocks];
        for (auto& p : prog)
            p = start;
        uint64_t ent[gcs::kServerSlots];
        for (auto& e : ent)
            e = (uint64_t)start << 32;   // as for the slots: never newer than a request
        HIP_TRY(hipMemcpyAsync(dpub_->prog[k], prog, sizeof prog, hipMemcpyHostToDevice, stream_));
        HIP_TRY(hipMemcpyAsync(dpub_->ent[k], ent, sizeof ent, hipMemcpyHostToDevice, stream_));
        HIP_TRY(hipStreamSynchronize(stream_));
        mask_ |= 1u << k;
        *r = k;
        return GCS_OK;
    }

    // A context leaves (its requests all complete): the grid leaves too, and
    // the next request of another ring starts one without this ring.
    int leave(int r)
    {
        std::lock_guard<std::mutex> lk(mu_);
        int rc = stop_locked();
        mask_ &= ~(1u << r);
        return rc;
    }

    // Make sure a grid whose group for ring r has not begun to leave serves
    // it: start one if none runs or (a block of) r's group left.
    int ensure(int r)
    {
        if (running(r))
            return GCS_OK;
        std::lock_guard<std::mutex> lk(mu_);
        if (running(r))
            return GCS_OK;
        int rc = stop_locked();
        if (rc) return rc;
        return launch_locked();
    }

    bool running(int r) const
    {
        if (!launched_.load(std::memory_order_acquire))
            return false;
        const gcs::ServerMailbox& m = mb_->ring[r];
        for (int b = 0; b < gcs::kServerBlocks; b++)
            if (__atomic_load_n(&m.state[b].v, __ATOMIC_ACQUIRE) == 2)
                return false;
        return true;
    }

    // Ask the grid to leave and wait until it has (the exit path of a
    // request that got no answer).
    int stop()
    {
        std::lock_guard<std::mutex> lk(mu_);
        return stop_locked();
    }

    gcs::ServerMailbox* ring(int r) { return &mb_->ring[r]; }
    gcs::ServerReq* reqs(int r) { return rq_->req[r]; }
    const uint64_t (*prof_sums(int r) const)[gcs::kProfWords] { return rq_->prof[r]; }
    bool dev_mailbox() const { return dev_mailbox_; }
    bool prof() const { return prof_; }
    bool print() const { return print_; }
    double ticks_per_us() const { return ticks_per_us_; }

  private:
    int init(int device)
    {
        HIP_TRY(hipHostMalloc((void**)&mb_, sizeof(gcs::HubMailbox),
                              hipHostMallocCoherent | hipHostMallocMapped));
        std::memset(mb_, 0, sizeof(gcs::HubMailbox));
        HIP_TRY(hipHostGetDevicePointer((void**)&dmb_, mb_, 0));
        // The request lines: uncached device memory the host writes over the
        // BAR (default), so a poll reads HBM and puts nothing on the PCIe
        // link: a poll takes 0.64-0.68 us at 1-16 rings, against 1.8 -> 8 us
        // over PCIe in pinned host memory (GCS_SERVER_MAILBOX=host, or when
        // the allocation fails).  The records stay in host
        // memory either way.
        const char* mbx = std::getenv("GCS_SERVER_MAILBOX");
        if (!mbx || std::strcmp(mbx, "host") != 0) {
            if (hipExtMallocWithFlags((void**)&rq_, sizeof(gcs::HubReqs),
                                      hipDeviceMallocUncached) == hipSuccess) {
                drq_ = rq_;
                dev_mailbox_ = true;
            } else {
                (void)hipGetLastError();
                rq_ = nullptr;
            }
        }
        if (!rq_) {
            HIP_TRY(hipHostMalloc((void**)&rq_, sizeof(gcs::HubReqs),
                                  hipHostMallocCoherent | hipHostMallocMapped));
            HIP_TRY(hipHostGetDevicePointer((void**)&drq_, rq_, 0));
        }
        std::memset(rq_, 0, sizeof(gcs::HubReqs));
        if (dev_mailbox_)
            _mm_sfence();
        // GCS_SERVER_ACQUIRE (A/B knobs, gcs_internal.h kServerAcq*): agent =
        // every acquire at agent scope (frames in registered host memory may
        // then be read from a stale L2 line); none = no acquire for frames in
        // device staging or in an uncached registered region (A/B only: a
        // CU's L1 may still hold an earlier request's lines).  Default: agent
        // scope for device frames, the L1 invalidate for uncached host frames,
        // system scope for other host frames.
        const char* acq = std::getenv("GCS_SERVER_ACQUIRE");
        opts_ = !acq                         ? 0u
                : std::strcmp(acq, "agent") == 0 ? gcs::kServerAcqAgent
                : std::strcmp(acq, "none") == 0  ? gcs::kServerAcqNone
                                                 : 0u;

        HIP_TRY(hipMalloc((void**)&dpub_, sizeof(gcs::HubPub)));
        HIP_TRY(hipMemset(dpub_, 0, sizeof(gcs::HubPub)));
        // the highest priority: a queue pool of its own, so the resident grid
        // holds back no context's launches behind it on a shared hardware queue
        int least = 0, greatest = 0;
        HIP_TRY(hipDeviceGetStreamPriorityRange(&least, &greatest));
        HIP_TRY(hipStreamCreateWithPriority(&stream_, hipStreamNonBlocking, greatest));
        int khz = 0;
        HIP_TRY(hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, device));
        ticks_per_us_ = khz > 0 ? khz / 1000.0 : 100.0;
        // GCS_SERVER_COUNTERS=1 (or GCS_SERVER_PROF): the grid build with
        // per-block phase counters (a clock read and a wait per phase,
        // gcs_server_stats_get's GPU figures), 1-3 us slower per burst than the
        // plain build.  GCS_SERVER_PROF also prints each ring's
        // figures at exit.  Process-wide.
        const char* ctr = std::getenv("GCS_SERVER_COUNTERS");
        print_ = std::getenv("GCS_SERVER_PROF") != nullptr;
        prof_ = (ctr && std::strcmp(ctr, "0") != 0) || print_;
        read_knobs();
        return GCS_OK;
    }

    // Read at each join (under mu_), so a process (a test) may change them
    // between contexts.
    void read_knobs()
    {
        // a group that leaves alone makes the next request of its ring restart
        // the whole grid: idle rings go cold instead (hot_ticks), and by
        // default only the lifetime ends the grid
        const char* e = std::getenv("GCS_SERVER_IDLE_US");
        idle_ticks_ = (uint64_t)((e ? std::atof(e) : 10000.0) * ticks_per_us_);
        e = std::getenv("GCS_SERVER_LIFE_US");
        // every ring waits for a relaunch: 10 ms (12 threads per GPU: 18 us
        // per burst, 23 us with 2 ms; the grid holds no other launch back)
        life_ticks_ = (uint64_t)((e ? std::atof(e) : 10000.0) * ticks_per_us_);
        // a ring without a request for this long goes cold: only the leader
        // block polls its host lines (0: never cold)
        e = std::getenv("GCS_SERVER_HOT_US");
        // (at least 2 us: a block must stay hot from seeing its request to
        // reading its lines, or it never serves)
        const double hot_us = e ? (std::atof(e) > 0 ? std::max(std::atof(e), 2.0) : 0.0) : 20.0;
        hot_ticks_ = hot_us > 0 ? (uint64_t)(hot_us * ticks_per_us_) : ~0ull;
        // ... and stays hot longer, up to this, while its requests come in
        // short gaps (3 x the gap: a thread bursting every 50 us stays hot)
        e = std::getenv("GCS_SERVER_HOT_MAX_US");
        const double hot_max_us = e ? std::atof(e) : 200.0;
        hot_max_ticks_ = hot_us > 0 ? (uint64_t)(std::max(hot_us, hot_max_us) * ticks_per_us_)
                                    : ~0ull;
        // extra ~2 us naps between the polls of a block with no hot ring, and
        // of a hot one (an A/B knob for the PCIe cost of hot polling)
        // (clamped to [0, 0xFFFF]: a negative value must not become a huge
        // unsigned nap count that stops the grid from serving)
        e = std::getenv("GCS_SERVER_COLD_NAPS");
        naps_ = e ? (uint32_t)std::clamp(std::atoi(e), 0, 0xFFFF) : 0u;
        e = std::getenv("GCS_SERVER_HOT_NAPS");
        naps_ |= (e ? (uint32_t)std::clamp(std::atoi(e), 0, 0xFFFF) : 0u) << 16;
    }

    // Every block ends within life_ticks of its start (or at the exit
    // command); the stream sync then confirms the grid has drained.
    int stop_locked()
    {
        if (!launched_.load(std::memory_order_relaxed))
            return GCS_OK;
        __atomic_store_n(&rq_->cmd.v, 1u, __ATOMIC_RELEASE);
        if (dev_mailbox_)
            _mm_sfence();                 // write-combined over the BAR: out now
        HIP_TRY(hipStreamSynchronize(stream_));
        launched_.store(false, std::memory_order_release);
        return GCS_OK;
    }

    // One group of kServerBlocks blocks per ring in use.
    int launch_locked()
    {
        if (mask_ == 0)
            return GCS_OK;
        int groups = 0;
        for (int k = 0; k < gcs::kHubRings; k++) {
            if (!((mask_ >> k) & 1u))
                continue;
            for (auto& st : mb_->ring[k].state)
                __atomic_store_n(&st.v, 0u, __ATOMIC_RELAXED);
            ring_of_[groups++] = (uint32_t)k;
        }
        __atomic_store_n(&rq_->cmd.v, 0u, __ATOMIC_RELEASE);
        if (dev_mailbox_)
            _mm_sfence();
        HIP_TRY(hipMemsetAsync(dpub_->exit, 0, sizeof dpub_->exit, stream_));
        // ring_of_ is only rewritten under mu_ after the previous grid left and
        // this copy completed (stop_locked synchronises the stream)
        HIP_TRY(hipMemcpyAsync(dpub_->ring_of, ring_of_, groups * sizeof(uint32_t),
                               hipMemcpyHostToDevice, stream_));
        HIP_TRY(gcs::launch_burst_server(dmb_, drq_, dpub_, groups, idle_ticks_, life_ticks_,
                                         hot_ticks_, hot_max_ticks_, kMaxPolls, naps_, opts_,
                                         prof_, stream_));
        launched_.store(true, std::memory_order_release);
        return GCS_OK;
    }

    static constexpr uint32_t kMaxPolls = 1u << 22;   // hard bound beside the clock
    static constexpr int kMaxDevices = 64;
    static std::mutex& registry_mu()
    {
        static std::mutex m;
        return m;
    }
    static ServerHub** registry()
    {
        static ServerHub* hubs[kMaxDevices] = {};
        return hubs;
    }
    std::mutex mu_;
    gcs::HubMailbox* mb_ = nullptr;       // host view
    gcs::HubMailbox* dmb_ = nullptr;      // device view
    gcs::HubReqs* rq_ = nullptr;          // request lines, host view
    gcs::HubReqs* drq_ = nullptr;         // ... device view
    bool dev_mailbox_ = false;            // rq_ is device memory (write-combined BAR)
    uint32_t opts_ = 0;                   // launch_burst_server opts
    gcs::HubPub* dpub_ = nullptr;         // device memory
    hipStream_t stream_ = nullptr;
    uint32_t mask_ = 0;                   // rings in use
    std::atomic<bool> launched_{false};
    uint64_t idle_ticks_ = 0, life_ticks_ = 0, hot_ticks_ = 0, hot_max_ticks_ = 0;
    uint32_t ring_of_[gcs::kHubRings] = {};
    uint32_t naps_ = 0;                   // cold naps | hot naps << 16
    bool prof_ = false, print_ = false;
    double ticks_per_us_ = 100.0;
};

// One context's request ring.  post() returns at once; wait(q) completes
// every request up to q, in order.  Used by one thread at a time (the
// context's).
class BurstServer {
  public:
    ~BurstServer() { (void)shutdown(); }

    // Complete what is posted, then leave the hub (its grid stops; another
    // ring's next request starts a fresh one).  The first failure is returned
    // -- gcs_ctx_destroy and gcs_ctx_set_burst_server(ctx, 0) report it -- so
    // a device fault at teardown is charged to this context, not to the next
    // caller that happens to check.
    int shutdown()
    {
        if (!hub_ || r_ < 0)
            return GCS_OK;
        print_stats();
        const int rc = wait(posted_);
        const int rc2 = hub_->leave(r_);
        r_ = -1;
        return rc ? rc : rc2;
    }

    void print_stats() const
    {
        if (prof_n_ && hub_->print()) {
            gcs_server_stats st;
            stats(&st);
            std::fprintf(stderr,
                         "[gcs burst server] %llu requests: request writes %.2f us; post->done "
                         "%.2f us, GPU span %.2f us (%llu measured); per block: poll %.2f us "
                         "(seen %.2f), acquire %.2f, frames %.2f, records %.2f, release %.2f; "
                         "seen skew %.2f, slowest block %.2f, cold %.2f\n",
                         (unsigned long long)st.requests, prof_write_ / prof_n_,
                         st.post_to_done_us, st.gpu_span_us, (unsigned long long)prof_n_,
                         st.poll_us, st.seen_poll_us, st.acquire_us, st.frames_us,
                         st.records_us, st.release_us, st.seen_skew_us, st.block_serve_us,
                         st.cold_frac);
        }
    }

    int init(int device)
    {
        hub_ = ServerHub::get(device);
        if (!hub_) {
            std::snprintf(g_hip_err, sizeof g_hip_err, "burst server: hub setup failed");
            return GCS_EHIP;
        }
        // test-only (tests/test_gpu_host.py): start the request numbers near a
        // 16-bit tag or 32-bit wrap instead of after 65k real bursts
        if (const char* s = std::getenv("GCS_SERVER_SEQ_START"))
            posted_ = done_ = (uint32_t)std::strtoul(s, nullptr, 0);
        int rc = hub_->join(done_, &r_);
        if (rc) return rc;
        mb_ = hub_->ring(r_);
        rq_ = hub_->reqs(r_);
        dev_ = hub_->dev_mailbox();
        read_wait_knobs();
        return GCS_OK;
    }

    // Post one request (n <= gcs::kSlotFrames): frames at device address
    // `frames` (bytes, a multiple of 16), frame i at off[i], len[i] bytes.
    // When it completes (wait), the verdicts / statuses go to code[] and, for a
    // fill, the checks to csum[]: both must stay valid until then.
    // in_place: the kernel writes the frames themselves (host memory), so
    // completion also waits for the serving blocks' release + ack; otherwise
    // the tagged result records alone complete it.
    // where: where the frames live, as line A's mode bits (gcs_internal.h):
    // kModeDevFrames (device staging: an agent-scope acquire makes them
    // visible), kModeUncachedFrames (a region registered uncached: no cache
    // above the GPU's L1 holds its lines), or 0 (pinned host memory).
    int post(uint8_t* frames, uint64_t bytes, const uint64_t* off, const uint16_t* len,
             uint32_t n, bool compute, uint32_t flags, uint8_t* code, uint32_t* csum,
             bool in_place, uint32_t where, uint32_t* ticket)
    {
        const uint64_t fa = reinterpret_cast<uint64_t>(frames);
        if ((fa & ~gcs::kAddrMask) || n > (uint32_t)gcs::kSlotFrames) {
            std::snprintf(g_hip_err, sizeof g_hip_err,
                          "burst server: frames above 2^48 or more than one request's frames");
            return GCS_EINVAL;
        }
        const uint32_t q = gcs::server_next(posted_);
        Req& r = req_[q % gcs::kServerSlots];
        if (r.pending) {                  // the slot's previous request must be done
            int rc = wait(r.q);
            if (rc) return rc;
        }
        int rc = hub_->ensure(r_);
        if (rc) return rc;
        gcs::ServerReq& sl = rq_[q % gcs::kServerSlots];
        const auto tw = std::chrono::steady_clock::now();
        std::memset(mb_->res[q % gcs::kServerSlots].rec, 0, n * sizeof(uint64_t));   // no record
                                                                                     // of an older request
        const uint32_t mode = (compute ? 1u : 0u) | (flags << 1) |
                              (where & (gcs::kModeDevFrames | gcs::kModeUncachedFrames));
        // every line carries the request in both 8 B halves (gcs_internal.h):
        // the tag in the top 16 bits of the address / offset and beside n
        const uint64_t tag = gcs::server_tag(q);
        auto tagged = [&](uint64_t a) {
            // an offset past 2^48 cannot lie inside the frames (a region is
            // < 64 GiB): it is kept out of bounds, so the kernel flags the frame
            return (a > gcs::kAddrMask ? gcs::kAddrMask : a) | tag << gcs::kTagShift;
        };
        const uint64_t fb = fa | tag << gcs::kTagShift;
        const uint32_t na = n | (uint32_t)tag << 16;
        if (dev_) {
            // Device memory over the BAR, write-combined: each 16 B line goes
            // out as ONE aligned 16 B store, the descriptors and line B first,
            // then (sfence) line A, then sfence again so the request leaves
            // the write-combining buffers now.
            for (uint32_t i = 0; i < n; i++) {
                const uint64_t o = tagged(off[i]);
                _mm_store_si128(reinterpret_cast<__m128i*>(&sl.desc[i]),
                                _mm_set_epi32((int)q, (int)len[i], (int)(uint32_t)(o >> 32),
                                              (int)(uint32_t)o));
            }
            _mm_store_si128(reinterpret_cast<__m128i*>(&sl.b),
                            _mm_set_epi32((int)q, (int)(uint32_t)(bytes / 16),
                                          (int)(uint32_t)(fb >> 32), (int)(uint32_t)fb));
            _mm_sfence();
            r = Req{q, n, compute, in_place, true, code, csum, 0, std::chrono::steady_clock::now()};
            _mm_store_si128(reinterpret_cast<__m128i*>(&sl.a),
                            _mm_set_epi32((int)mode, (int)na, 0, (int)q));
            _mm_sfence();
        } else {
            // each 16 B line: its fields, then its seq (x86 keeps the order)
            for (uint32_t i = 0; i < n; i++) {
                gcs::ServerDesc& d = sl.desc[i];
                d.off = tagged(off[i]);
                d.len = len[i];
                __atomic_store_n(&d.seq, q, __ATOMIC_RELEASE);
            }
            sl.b.frames = fb;
            sl.b.bytes16 = (uint32_t)(bytes / 16);
            __atomic_store_n(&sl.b.seq, q, __ATOMIC_RELEASE);
            sl.a.n = na;
            sl.a.mode = mode;
            sl.a.cmd = 0;
            r = Req{q, n, compute, in_place, true, code, csum, 0, std::chrono::steady_clock::now()};
            __atomic_store_n(&sl.a.seq, q, __ATOMIC_RELEASE);
        }
        if (hub_->prof())
            prof_write_ += std::chrono::duration<double, std::micro>(r.t0 - tw).count();
        posted_ = q;
        if (ticket) *ticket = q;
        return GCS_OK;
    }

    // Complete every posted request up to and including q, in order.
    int wait(uint32_t q)
    {
        while ((int32_t)(q - done_) > 0 && done_ != posted_) {
            const uint32_t r = gcs::server_next(done_);
            int rc = complete(req_[r % gcs::kServerSlots]);
            if (rc) return rc;
            done_ = r;
        }
        return GCS_OK;
    }

    uint32_t posted() const { return posted_; }

    // Serve one batch (n <= gcs::kServerMaxFrames) and return when it is done.
    int serve(uint8_t* frames, uint64_t bytes, const uint64_t* off, const uint16_t* len,
              uint32_t n, bool compute, uint32_t flags, uint8_t* code, uint32_t* csum,
              bool in_place, uint32_t where)
    {
        uint32_t q = done_;
        for (uint32_t k = 0; k < n; k += gcs::kSlotFrames) {
            const uint32_t m = std::min<uint32_t>(gcs::kSlotFrames, n - k);
            int rc = post(frames, bytes, off + k, len + k, m, compute, flags,
                          code ? code + k : nullptr, csum ? csum + k : nullptr, in_place,
                          where, &q);
            if (rc) return rc;
        }
        return wait(q);
    }

    // Complete what is posted (the grid stays for the other rings).
    int stop() { return wait(posted_); }

  private:
    struct Req {
        uint32_t q, n;
        bool compute, in_place, pending;
        uint8_t* code;
        uint32_t* csum;
        uint32_t have;                               // records [0, have) carry q
        std::chrono::steady_clock::time_point t0;    // posted
    };

    // One step of the host's wait for a request, `waited` into it.  Spin
    // (pause) first; past GCS_SERVER_SPIN_US, GCS_SERVER_WAIT=yield gives the
    // CPU to another runnable thread at each step (sched_yield), and =sleep
    // sleeps GCS_SERVER_SLEEP_NS per step (with the thread's timer slack at
    // 1 ns, set on first use): a thread that waits long stops burning the
    // CPU share (cgroup quota) the other mTCP threads of the host need.
    // Default: spin.
    void idle(std::chrono::steady_clock::duration waited)
    {
        if (wait_mode_ == kWaitSpin || waited < spin_) {
            __builtin_ia32_pause();
            return;
        }
        if (wait_mode_ == kWaitYield) {
            sched_yield();
            return;
        }
        if (!slack_set_) {
            (void)prctl(PR_SET_TIMERSLACK, 1UL, 0UL, 0UL, 0UL);
            slack_set_ = true;
        }
        const struct timespec ts = {0, sleep_ns_};
        nanosleep(&ts, nullptr);
    }

    void read_wait_knobs()
    {
        const char* e = std::getenv("GCS_SERVER_WAIT");
        wait_mode_ = !e                            ? kWaitSpin
                     : std::strcmp(e, "yield") == 0 ? kWaitYield
                     : std::strcmp(e, "sleep") == 0 ? kWaitSleep
                                                    : kWaitSpin;
        e = std::getenv("GCS_SERVER_SPIN_US");
        spin_ = std::chrono::nanoseconds((long)(1000.0 * (e ? std::max(0.0, std::atof(e)) : 4.0)));
        e = std::getenv("GCS_SERVER_SLEEP_NS");
        sleep_ns_ = e ? std::clamp(std::atol(e), 1L, 1000000L) : 1000L;
        e = std::getenv("GCS_SERVER_PRESLEEP_NS");
        presleep_ns_ = e ? std::clamp(std::atol(e), 0L, 100000L) : 0L;
    }

    // GCS_SERVER_PRESLEEP_NS: sleep this long right after posting, before the
    // spin -- no request completes sooner than the grid's round trip, so a
    // thread that sleeps through part of it gives that CPU time back to the
    // other mTCP threads of a CPU quota without waiting longer itself, as long
    // as its wake-up comes before the records (timer slack 1 ns).
    void presleep()
    {
        if (!slack_set_) {
            (void)prctl(PR_SET_TIMERSLACK, 1UL, 0UL, 0UL, 0UL);
            slack_set_ = true;
        }
        const struct timespec ts = {0, presleep_ns_};
        nanosleep(&ts, nullptr);
    }

    // Wait until request r is done (its records, and for an in-place request
    // the serving blocks' acks), starting a grid when the last one left first.
    int complete(Req& r)
    {
        const uint64_t tag = (uint64_t)(r.q & 0xFFFFu) << 48;
        gcs::ServerRes& sl = mb_->res[r.q % gcs::kServerSlots];
        const int nb = (int)std::min<uint32_t>(gcs::kServerBlocks,
                                               (r.n + gcs::kServerFPB - 1) / gcs::kServerFPB);
        const auto t0 = std::chrono::steady_clock::now();
        if (presleep_ns_ && r.have == 0 && r.n &&
            (__atomic_load_n(&sl.rec[0], __ATOMIC_ACQUIRE) >> 48) != (tag >> 48))
            presleep();
        for (;;) {
            while (r.have < r.n &&
                   (__atomic_load_n(&sl.rec[r.have], __ATOMIC_ACQUIRE) >> 48) == (tag >> 48))
                r.have++;
            bool all = r.have == r.n;
            if (all && r.in_place)
                for (int k = 0; k < nb; k++) {
                    // an ack counts only inside [r.q, posted_]: one past the
                    // last request posted is stale (a ring joined with old
                    // acks, GCS_FAULT_INJECT=ack_skew) and proves nothing
                    // about r's writes
                    const int b = gcs::server_block(r.q, (uint32_t)k * gcs::kServerFPB);
                    const uint32_t ak = __atomic_load_n(&mb_->ack[b].v, __ATOMIC_ACQUIRE);
                    if ((int32_t)(ak - r.q) < 0 || (int32_t)(posted_ - ak) < 0)
                        all = false;
                }
            if (all)
                break;
            if (!hub_->running(r_)) {
                // the grid left (or is leaving) before serving r: a fresh grid
                // resumes each block where it stopped
                int rc = hub_->ensure(r_);
                if (rc) return rc;
                continue;
            }
            const auto now = std::chrono::steady_clock::now();
            if (now - t0 > std::chrono::seconds(2)) {
                (void)hub_->stop();
                std::snprintf(g_hip_err, sizeof g_hip_err, "burst server: no answer in 2 s");
                return GCS_EHIP;
            }
            idle(now - t0);
        }
        for (uint32_t i = 0; i < r.n; i++) {
            const uint64_t v = sl.rec[i];
            if (r.code) r.code[i] = (uint8_t)(v >> 32);
            if (r.compute && r.csum) r.csum[i] = (uint32_t)v;
        }
        r.pending = false;
        const double total = std::chrono::duration<double, std::micro>(
                                 std::chrono::steady_clock::now() - r.t0).count();
        n_done_++;
        total_us_ += total;
        if (hub_->prof() && r.n) {
            // phase counters: the request's GPU span, from the first serving
            // block's poll that saw it to the last one's records stored (GPU
            // wall clock).  A block writes its marks after its records, so
            // wait briefly for each serving block's tag; a block that has
            // already moved on to a later request is left out.
            bool first = true;
            uint64_t seen = 0, seen_max = 0, rec = 0, serve = 0;
            uint64_t seen_b[gcs::kServerBlocks] = {};
            bool have_b[gcs::kServerBlocks] = {};
            const auto tp = std::chrono::steady_clock::now();
            for (int k = 0; k < nb; k++) {
                const int b = gcs::server_block(r.q, (uint32_t)k * gcs::kServerFPB);
                const __m128i* mp = reinterpret_cast<const __m128i*>(&mb_->mark[b][0]);
                alignas(16) uint32_t mk[4];
                int32_t d;
                for (;;) {
                    asm volatile("" ::: "memory");   // the grid writes it: reload
                    _mm_store_si128(reinterpret_cast<__m128i*>(mk), _mm_load_si128(mp));
                    d = (int32_t)(mk[3] - r.q);
                    if (d >= 0 || std::chrono::steady_clock::now() - tp >
                                      std::chrono::microseconds(200))
                        break;
                    __builtin_ia32_pause();
                }
                if (d != 0)
                    continue;
                const uint64_t s0 = (uint64_t)mk[0] | ((uint64_t)mk[1] << 32), r0 = s0 + mk[2];
                if (first) {
                    seen = seen_max = s0;
                    rec = r0;
                    first = false;
                }
                seen = std::min(seen, s0);
                seen_max = std::max(seen_max, s0);
                rec = std::max(rec, r0);
                serve = std::max<uint64_t>(serve, mk[2]);
                seen_b[b] = s0;
                have_b[b] = true;
            }
            if (!first && rec > seen) {
                const double tu = hub_->ticks_per_us();
                prof_n_++;
                prof_span_ += (double)(rec - seen) / tu;
                prof_skew_ += (double)(seen_max - seen) / tu;
                prof_serve_ += (double)serve / tu;
                for (int b = 0; b < gcs::kServerBlocks; b++)
                    if (have_b[b]) {
                        late_[b] += (double)(seen_b[b] - seen) / tu;
                        late_n_[b]++;
                    }
                // host clock vs GPU clock: d1 = seen - post and d2 = done -
                // rec each carry the clocks' unknown offset with opposite
                // signs; the smallest d1 stands for the fastest post -> seen
                const double post_us = std::chrono::duration<double, std::micro>(
                                           r.t0.time_since_epoch()).count();
                const double done_us = post_us + total;
                const double d1 = seen / tu - post_us, d2 = done_us - rec / tu;
                d1_sum_ += d1;
                d2_sum_ += d2;
                d1_min_ = prof_n_ == 1 ? d1 : std::min(d1_min_, d1);
            }
        }
        return GCS_OK;
    }

  public:
    // gcs_server_stats_get: this ring's figures so far (GPU parts with
    // the counting build only, GCS_SERVER_COUNTERS).
    void stats(gcs_server_stats* st) const
    {
        std::memset(st, 0, sizeof *st);
        st->requests = n_done_;
        st->post_to_done_us = n_done_ ? total_us_ / n_done_ : 0.0;
        if (!hub_->prof())
            return;
        st->gpu_span_us = prof_n_ ? prof_span_ / prof_n_ : 0.0;
        st->seen_wait_us = prof_n_ ? d1_sum_ / prof_n_ - d1_min_ : 0.0;
        st->after_gpu_us = prof_n_ ? d2_sum_ / prof_n_ + d1_min_ : 0.0;
        st->seen_skew_us = prof_n_ ? prof_skew_ / prof_n_ : 0.0;
        st->block_serve_us = prof_n_ ? prof_serve_ / prof_n_ : 0.0;
        // the sums live beside the request lines (device memory by default:
        // read over the BAR, a few hundred slow loads, only here)
        uint64_t sum[gcs::kProfWords] = {};
        const uint64_t (*pr)[gcs::kProfWords] = hub_->prof_sums(r_);
        for (int b = 0; b < gcs::kServerBlocks; b++)
            for (int k = 0; k < gcs::kProfWords; k++)
                sum[k] += k == gcs::kProfMaxRtt ? 0 : __atomic_load_n(&pr[b][k], __ATOMIC_RELAXED);
        const double tu = hub_->ticks_per_us();
        const double nreq = sum[gcs::kProfN] ? (double)sum[gcs::kProfN] : 1.0;
        st->block_requests = sum[gcs::kProfN];
        st->polls = sum[gcs::kProfPolls];
        st->poll_us = sum[gcs::kProfPolls] ? sum[gcs::kProfPollRtt] / tu / sum[gcs::kProfPolls]
                                           : 0.0;
        st->seen_poll_us = sum[gcs::kProfSeenRtt] / tu / nreq;
        st->acquire_us = sum[gcs::kProfAcq] / tu / nreq;
        st->frames_us = sum[gcs::kProfFrames] / tu / nreq;
        st->records_us = sum[gcs::kProfRecs] / tu / nreq;
        st->release_us = sum[gcs::kProfRel] / tu / nreq;
        st->cold_frac = sum[gcs::kProfCold] / nreq;
        st->slow_polls_2us = sum[gcs::kProfSlow2];
        st->slow_polls_5us = sum[gcs::kProfSlow5];
        st->torn_polls = sum[gcs::kProfTorn];
        uint64_t mx = 0;
        for (int b = 0; b < gcs::kServerBlocks; b++)
            mx = std::max<uint64_t>(mx, __atomic_load_n(&pr[b][gcs::kProfMaxRtt],
                                                        __ATOMIC_RELAXED));
        st->max_poll_us = mx / tu;
        for (int b = 0; b < gcs::kServerBlocks; b++)
            st->late_us[b] = late_n_[b] ? late_[b] / late_n_[b] : 0.0;
    }

  private:

    enum { kWaitSpin = 0, kWaitYield = 1, kWaitSleep = 2 };
    int wait_mode_ = kWaitSpin;           // GCS_SERVER_WAIT (idle)
    std::chrono::nanoseconds spin_{4000};
    long sleep_ns_ = 1000;
    long presleep_ns_ = 0;                // GCS_SERVER_PRESLEEP_NS (complete)
    bool slack_set_ = false;
    ServerHub* hub_ = nullptr;
    int r_ = -1;                          // ring index in the hub
    gcs::ServerMailbox* mb_ = nullptr;    // this ring (host view)
    gcs::ServerReq* rq_ = nullptr;        // its request lines (host view)
    bool dev_ = false;                    // ... in device memory, over the BAR
    uint32_t posted_ = 0;                 // last request posted
    uint32_t done_ = 0;                   // last request completed (all before it too)
    Req req_[gcs::kServerSlots] = {};
    uint64_t n_done_ = 0, prof_n_ = 0;
    double total_us_ = 0, prof_span_ = 0, prof_skew_ = 0, prof_serve_ = 0, prof_write_ = 0;
    double late_[gcs::kServerBlocks] = {};
    double d1_sum_ = 0, d2_sum_ = 0, d1_min_ = 0;
    uint64_t late_n_[gcs::kServerBlocks] = {};
};

}  // namespace

struct gcs_ctx {
    int device = 0;
    hipStream_t stream = nullptr;
    // RSS steering (gcs_ctx_set_rss), see set_rss_params
    uint32_t rss_key[4] = {0x05050505u, 0x05050505u, 0x05050505u, 0x05050505u};
    uint32_t rss_nq = 1, rss_magic = 0, rss_endian = 0;
    uint32_t max_frames = 0;   // per slot
    uint64_t max_bytes = 0;    // per slot
    uint64_t direct_max = 0;   // host batches up to this many staged bytes: direct mode
    bool direct_spread = true; // direct mode 8 frames per block (server / k_desc_rec), not k_desc_mixed
    Slot slot[kSlots];
    std::unique_ptr<GatherPool> pool;
    std::unique_ptr<BurstServer> server;   // gcs_ctx_set_burst_server / GCS_BURST_SERVER

    // gcs_compute_ptrs_async: one record per server slot (request q lives in
    // slot q % kServerSlots), with its own pinned staging for pageable frames
    struct AsyncReq {
        bool pending = false;
        bool staged = false;
        bool compute = true;                // a TX fill, or an RX verify
        bool cancelled = false;             // a failed wait dropped it: the next wait
                                            // covering it reports the failure
        uint32_t flags = 0;                 // verify: GCS_VF_ZERO_BAD_TCP_CHECK (applied by the host)
        uint32_t q = 0, n = 0;
        uint8_t* status = nullptr;          // the caller's outputs (nullable)
        uint32_t* csums = nullptr;
        std::vector<uint8_t*> ptrs;         // the caller's frames (staged: scatter target)
        std::vector<uint16_t> lens;
        std::vector<uint64_t> off;          // descriptors as posted
        std::vector<uint16_t> dlen;
        std::vector<uint8_t> st;            // results, written by the server
        std::vector<uint32_t> cs;
        uint8_t* h_stage = nullptr;         // pinned staging (kAsyncStageBytes)
        uint8_t* d_stage = nullptr;         // its device view
        bool stage_dev = false;             // staging is device memory (hipFree)
    };
    // Bursts from pageable memory are staged in fine-grained device memory
    // written over the BAR (default; GCS_ASYNC_STAGE / GCS_DIRECT_STAGE=host
    // for pinned host staging): the GPU then reads HBM instead of PCIe.  A
    // failed device allocation turns it off for the context (host staging).
    bool async_stage_dev = true;            // gcs_*_ptrs_async
    bool direct_stage_dev = true;           // direct-mode (burst) host batches
    // Async bursts from a registered region are staged like pageable ones
    // when staging is device memory: the GPU reads HBM, not the region over
    // PCIe (64 x 1500 B TX, tools/tx_async_probe.py: send_pkts blocked
    // 5.3-5.5 vs 7.3-7.6 us in place).  GCS_ASYNC_REGISTERED=inplace reads
    // the region in place.
    bool async_reg_stage = true;
    // test-only: GCS_FAULT_INJECT was set (to anything) when the context was
    // made, so the per-burst entry points look up its value per call; an
    // unarmed context never reads the environment on the burst path
    bool faults = false;
    AsyncReq areq[gcs::kServerSlots];

    // Copy work for `count` frames / `bytes` bytes: inline when small, else
    // spread over the gather pool.
    void gather_run(uint32_t count, uint64_t bytes,
                    const std::function<void(uint32_t, uint32_t)>& fn)
    {
        const int t = GatherPool::threads();
        if (t <= 1 || bytes < (1u << 20) || count < 64) {
            fn(0, count);
            return;
        }
        if (!pool) {
            if (fault("gather_alloc"))
                throw std::bad_alloc();
            pool.reset(new GatherPool());
        }
        pool->run(count, (uint32_t)std::min<uint64_t>(4ull * t, count), fn);
    }
};

namespace {

struct DeviceGuard {
    int prev = -1;
    explicit DeviceGuard(int dev)
    {
        if (hipGetDevice(&prev) != hipSuccess)
            prev = -1;
        if (prev != dev)
            (void)hipSetDevice(dev);
    }
    ~DeviceGuard()
    {
        if (prev >= 0)
            (void)hipSetDevice(prev);
    }
};

hipStream_t pick_stream(gcs_ctx* ctx, void* stream)
{
    return stream ? reinterpret_cast<hipStream_t>(stream) : ctx->stream;
}

// Teardown keeps going past a failure (everything is released) and reports
// the first one: rc stays the first non-OK status.
void keep_first(int& rc, hipError_t e, const char* what)
{
    if (e != hipSuccess && rc == GCS_OK)
        rc = hip_fail(e, what);
}

int free_slot(Slot& s)
{
    int rc = GCS_OK;
    if (s.stream) keep_first(rc, hipStreamSynchronize(s.stream), "slot stream sync");
    if (s.h_frames) keep_first(rc, hipHostFree(s.h_frames), "hipHostFree");
    if (s.h_off) keep_first(rc, hipHostFree(s.h_off), "hipHostFree");
    if (s.h_len) keep_first(rc, hipHostFree(s.h_len), "hipHostFree");
    if (s.h_code) keep_first(rc, hipHostFree(s.h_code), "hipHostFree");
    if (s.h_csum) keep_first(rc, hipHostFree(s.h_csum), "hipHostFree");
    if (s.h_hash) keep_first(rc, hipHostFree(s.h_hash), "hipHostFree");
    if (s.h_queue) keep_first(rc, hipHostFree(s.h_queue), "hipHostFree");
    if (s.h_rec) keep_first(rc, hipHostFree(s.h_rec), "hipHostFree");
    if (s.d_hash) keep_first(rc, hipFree(s.d_hash), "hipFree");
    if (s.d_queue) keep_first(rc, hipFree(s.d_queue), "hipFree");
    if (s.d_frames) keep_first(rc, hipFree(s.d_frames), "hipFree");
    if (s.d_off) keep_first(rc, hipFree(s.d_off), "hipFree");
    if (s.d_len) keep_first(rc, hipFree(s.d_len), "hipFree");
    if (s.v_frames) keep_first(rc, hipFree(s.v_frames), "hipFree");
    if (s.d_code) keep_first(rc, hipFree(s.d_code), "hipFree");
    if (s.d_csum) keep_first(rc, hipFree(s.d_csum), "hipFree");
    if (s.done) keep_first(rc, hipEventDestroy(s.done), "hipEventDestroy");
    if (s.stream) keep_first(rc, hipStreamDestroy(s.stream), "hipStreamDestroy");
    s = Slot();
    return rc;
}

int alloc_slot(Slot& s, uint32_t frames, uint64_t bytes)
{
    HIP_TRY(hipStreamCreateWithFlags(&s.stream, hipStreamNonBlocking));
    HIP_TRY(hipEventCreateWithFlags(&s.done, hipEventDisableTiming));
    HIP_TRY(hipHostMalloc((void**)&s.h_frames, bytes, hipHostMallocDefault));
    HIP_TRY(hipHostMalloc((void**)&s.h_off, frames * sizeof(uint64_t), hipHostMallocDefault));
    HIP_TRY(hipHostMalloc((void**)&s.h_len, frames * sizeof(uint16_t), hipHostMallocDefault));
    HIP_TRY(hipHostMalloc((void**)&s.h_code, frames, hipHostMallocDefault));
    HIP_TRY(hipHostMalloc((void**)&s.h_csum, frames * sizeof(uint32_t), hipHostMallocDefault));
    HIP_TRY(hipMalloc((void**)&s.d_frames, bytes));
    HIP_TRY(hipMalloc((void**)&s.d_off, frames * sizeof(uint64_t)));
    HIP_TRY(hipMalloc((void**)&s.d_len, frames * sizeof(uint16_t)));
    HIP_TRY(hipMalloc((void**)&s.d_code, frames));
    HIP_TRY(hipMalloc((void**)&s.d_csum, frames * sizeof(uint32_t)));
    HIP_TRY(hipHostMalloc((void**)&s.h_hash, frames * sizeof(uint32_t), hipHostMallocDefault));
    HIP_TRY(hipHostMalloc((void**)&s.h_queue, frames * sizeof(uint16_t), hipHostMallocDefault));
    HIP_TRY(hipHostMalloc((void**)&s.h_rec, frames * sizeof(uint64_t), hipHostMallocDefault));
    HIP_TRY(hipMalloc((void**)&s.d_hash, frames * sizeof(uint32_t)));
    HIP_TRY(hipMalloc((void**)&s.d_queue, frames * sizeof(uint16_t)));
    HIP_TRY(hipHostGetDevicePointer((void**)&s.m_frames, s.h_frames, 0));
    HIP_TRY(hipHostGetDevicePointer((void**)&s.m_off, s.h_off, 0));
    HIP_TRY(hipHostGetDevicePointer((void**)&s.m_len, s.h_len, 0));
    HIP_TRY(hipHostGetDevicePointer((void**)&s.m_code, s.h_code, 0));
    HIP_TRY(hipHostGetDevicePointer((void**)&s.m_csum, s.h_csum, 0));
    HIP_TRY(hipHostGetDevicePointer((void**)&s.m_hash, s.h_hash, 0));
    HIP_TRY(hipHostGetDevicePointer((void**)&s.m_queue, s.h_queue, 0));
    HIP_TRY(hipHostGetDevicePointer((void**)&s.m_rec, s.h_rec, 0));
    return GCS_OK;
}

// The reference's built-in RSS key (rss.c:19-25).
constexpr uint8_t kDefaultRssKey[40] = {5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5,
                                        5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5,
                                        5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5, 5};

// RSS parameters as the kernels take them: key bits 0..127 as big-endian
// words (GetRSSHash only reaches key bit 127, rss.c:27-40) and the queue
// count with its division magic.
void set_rss_params(gcs_ctx* ctx, const uint8_t* key, uint32_t nq, uint32_t endian)
{
    for (int w = 0; w < 4; w++)
        ctx->rss_key[w] = ((uint32_t)key[4 * w] << 24) | ((uint32_t)key[4 * w + 1] << 16) |
                          ((uint32_t)key[4 * w + 2] << 8) | key[4 * w + 3];
    ctx->rss_nq = nq;
    ctx->rss_magic = nq > 1 ? (uint32_t)(((1ull << 32) + nq - 1) / nq) : 0u;
    ctx->rss_endian = endian;
}

gcs::Ext rss_ext(const gcs_ctx* ctx, uint32_t* hash, uint16_t* queue)
{
    return gcs::Ext{{ctx->rss_key[0], ctx->rss_key[1], ctx->rss_key[2], ctx->rss_key[3]}, hash,
                    queue, ctx->rss_nq, ctx->rss_magic, ctx->rss_endian};
}

// Write back the check fields the device computed for one TX frame.
void scatter_tx(uint8_t* f, uint32_t len, uint8_t st, uint32_t cs)
{
    if (st != GCS_TX_OK && st != GCS_TX_IP_ONLY && st != GCS_TX_BAD_TCPLEN)
        return;
    uint16_t ipc = (uint16_t)cs;
    std::memcpy(f + 24, &ipc, 2);                     // iph->check (ip_out.c:172)
    if (st == GCS_TX_OK) {
        uint32_t ts = 14 + 4u * (f[14] & 15u);
        uint16_t tcpc = (uint16_t)(cs >> 16);
        if (ts + 18 <= len)
            std::memcpy(f + ts + 16, &tcpc, 2);       // tcph->check (tcp_out.c:330)
    }
}

// Is [p, p + bytes) host memory the GPU can DMA from directly (hipHostMalloc'd
// or hipHostRegister'ed)?
bool is_pinned(const void* p, uint64_t bytes)
{
    if (!p || bytes == 0)
        return false;
    const uint8_t* q = static_cast<const uint8_t*>(p);
    for (const uint8_t* a : {q, q + bytes - 1}) {
        hipPointerAttribute_t at;
        if (hipPointerGetAttributes(&at, a) != hipSuccess) {
            (void)hipGetLastError();
            return false;
        }
        if (at.type != hipMemoryTypeHost)
            return false;
    }
    return true;
}

// Records of a direct-mode batch (k_desc_rec: csum | code << 32 per frame)
// into the slot's verdict / check arrays.
void unpack_records(const uint64_t* rec, uint32_t n, uint8_t* code, uint32_t* csum)
{
    for (uint32_t i = 0; i < n; i++) {
        const uint64_t v = rec[i];
        code[i] = (uint8_t)(v >> 32);
        csum[i] = (uint32_t)v;
    }
}

// tcp_in.c:1237 (tcph->check = 0 on a TCP checksum failure), on the host copy.
template <class FramePtr>
void zero_bad_tcp_checks(const uint8_t* code, uint32_t n, FramePtr frame_ptr, const uint16_t* len)
{
    for (uint32_t i = 0; i < n; i++) {
        if (code[i] != GCS_V_DROP_TCPCSUM)
            continue;
        uint8_t* f = frame_ptr(i);
        uint32_t ts = 14 + 4u * (f[14] & 15u);
        if (ts + 18 <= len[i])
            f[ts + 16] = f[ts + 17] = 0;
    }
}

// Host regions registered with gcs_host_register, with their device views.
// A host batch whose frames all lie in one of them can be served in place.
struct RegRegion {
    uint8_t* host;
    uint64_t bytes;
    uint8_t* dev;
    bool uncached;   // registered with hipExtHostRegisterUncached
};
std::mutex g_reg_mu;
std::vector<RegRegion> g_regions;

bool find_region(const void* p, RegRegion* out)
{
    const uint8_t* q = static_cast<const uint8_t*>(p);
    std::lock_guard<std::mutex> lk(g_reg_mu);
    for (const auto& r : g_regions)
        if (q >= r.host && q < r.host + r.bytes) {
            *out = r;
            return true;
        }
    return false;
}

// Generic staged host batch.  Frames are addressed by base + off[i] or by
// ptrs[i]; `compute` selects TX fill vs RX verify.
//
// Per slot (two slots alternate, so the host work of chunk k+1 overlaps the
// H2D / kernel / D2H of chunk k):
//   span mode    base is pinned and the chunk's offsets are 16 B-aligned and
//                increasing: ONE hipMemcpyAsync of [off[first], end) straight
//                from the caller's buffer (zero host copies);
//   gather mode  otherwise: frames are copied into the slot's pinned staging at
//                64 B-aligned slots (pslib.c:146), split over the context's
//                gather threads when the chunk is large.
int run_host_batch(gcs_ctx* ctx, uint8_t* base, const uint64_t* off, uint8_t* const* ptrs,
                   const uint16_t* len, uint32_t n, uint8_t* code, uint32_t* csums,
                   uint32_t flags, bool compute, uint32_t* hash = nullptr,
                   uint16_t* queue = nullptr)
{
    const bool classify = !compute && (hash || queue);
    if (!ctx || !len || (!base && !ptrs) || (base && !off))
        return GCS_EINVAL;
    if (!compute && !code)
        return GCS_EINVAL;
    if (ctx->max_frames == 0 || ctx->max_bytes == 0)
        return GCS_ERANGE;
    if (n == 0)
        return GCS_OK;
    DeviceGuard g(ctx->device);

    auto frame_ptr = [&](uint32_t i) -> uint8_t* { return ptrs ? ptrs[i] : base + off[i]; };

    // A frame that cannot fit one staging slot is refused before anything is
    // launched, so an ERANGE never leaves part of the batch processed.
    for (uint32_t i = 0; i < n; i++)
        if (frame_ptr(i) && (len[i] + kSlotAlign - 1) / kSlotAlign * kSlotAlign > ctx->max_bytes)
            return GCS_ERANGE;

    // Whatever way this call ends (error return, exception), no slot may stay
    // marked busy: a later call would otherwise drain this call's chunk into
    // its own output arrays.  On the normal path drain() has cleared them.
    struct SlotReset {
        gcs_ctx* c;
        ~SlotReset()
        {
            for (auto& s : c->slot)
                if (s.busy) {
                    if (!s.served)
                        (void)hipEventSynchronize(s.done);
                    s.busy = false;
                    s.served = false;
                    s.rec = false;
                }
        }
    } slot_reset{ctx};

    // span mode needs the whole referenced range pinned
    bool pinned = false;
    if (base) {
        uint64_t end = 0;
        for (uint32_t i = 0; i < n; i++)
            end = std::max<uint64_t>(end, off[i] + len[i]);
        pinned = is_pinned(base, end);
    }

    // Drain one slot: wait for its stream and hand its results back.
    auto drain = [&](Slot& s) -> int {
        if (!s.busy)
            return GCS_OK;
        if (!s.served)
            HIP_TRY(hipEventSynchronize(s.done));
        s.busy = false;
        s.served = false;
        if (s.rec) {
            unpack_records(s.h_rec, s.count, s.h_code, s.h_csum);
            s.rec = false;
        }
        if (!compute) {
            std::memcpy(code + s.first, s.h_code, s.count);
            if (hash)
                std::memcpy(hash + s.first, s.h_hash, s.count * sizeof(uint32_t));
            if (queue)
                std::memcpy(queue + s.first, s.h_queue, s.count * sizeof(uint16_t));
            return GCS_OK;
        }
        const uint32_t first = s.first;
        ctx->gather_run(s.count, (uint64_t)s.count * 256, [&, first](uint32_t lo, uint32_t hi) {
            for (uint32_t k = lo; k < hi; k++) {
                uint32_t i = first + k;
                uint8_t st = s.h_code[k];
                uint32_t cs = s.h_csum[k];
                if (code) code[i] = st;
                if (csums) csums[i] = cs;
                if (!(flags & GCS_CF_NO_INPLACE) && frame_ptr(i))
                    scatter_tx(frame_ptr(i), len[i], st, cs);
            }
        });
        return GCS_OK;
    };

    // In-place mode: a small batch whose frames all lie in ONE registered
    // region (e.g. an mbuf pool registered with gcs_host_register) at 16 B-
    // aligned addresses.  The kernel reads -- and for TX fills -- the frames
    // where they are, over PCIe: no gather into staging, no scatter back.
    if (!classify && !(flags & GCS_VF_ICMP) && n <= ctx->max_frames && ctx->direct_max) {
        RegRegion reg{};
        uint32_t first = 0;
        while (first < n && !frame_ptr(first))
            first++;
        bool ok = first < n && find_region(frame_ptr(first), &reg);
        uint64_t total = 0;
        for (uint32_t i = 0; ok && i < n; i++) {
            const uint8_t* p = frame_ptr(i);
            if (!p)
                continue;
            // inside the region's whole 16 B chunks (the kernel never reads past them)
            ok = p >= reg.host && (uint64_t)(p - reg.host) + len[i] <= (reg.bytes & ~15ull) &&
                 ((uintptr_t)p & 15) == 0;
            total += len[i];
        }
        if (ok && total <= ctx->direct_max) {
            Slot& s = ctx->slot[0];
            for (auto& sl : ctx->slot) {
                int rc = drain(sl);
                if (rc) return rc;
            }
            for (uint32_t i = 0; i < n; i++) {
                const uint8_t* p = frame_ptr(i);
                s.h_off[i] = p ? (uint64_t)(p - reg.host) : 0;
                s.h_len[i] = p ? len[i] : 0;
            }
            if (ctx->server && n <= (uint32_t)gcs::kServerMaxFrames) {
                int rc = ctx->server->serve(reg.dev, reg.bytes & ~15ull, s.h_off, s.h_len, n,
                                            compute, 0u, s.h_code, compute ? s.h_csum : nullptr,
                                            /*in_place=*/compute,
                                            reg.uncached ? gcs::kModeUncachedFrames : 0u);
                if (rc) return rc;
            } else {
                if (ctx->server) {
                    // this context's posted requests complete first (the grid
                    // runs on a queue of its own: it holds no launch back)
                    int rc = ctx->server->stop();
                    if (rc) return rc;
                }
                // results as whole 64 B lines of records (k_desc_rec)
                HIP_TRY(gcs::launch_desc_rec(reg.dev, reg.bytes & ~15ull, s.m_off, s.m_len, n,
                                             s.m_rec, compute, 0u, s.stream));
                HIP_TRY(hipEventRecord(s.done, s.stream));
                HIP_TRY(hipEventSynchronize(s.done));
                unpack_records(s.h_rec, n, s.h_code, s.h_csum);
            }
            if (code)
                std::memcpy(code, s.h_code, n);
            if (compute && csums)
                std::memcpy(csums, s.h_csum, n * sizeof(uint32_t));
            if (!compute && (flags & GCS_VF_ZERO_BAD_TCP_CHECK))
                zero_bad_tcp_checks(code, n, frame_ptr, len);
            return GCS_OK;
        }
    }

    uint32_t next = 0;
    int k = 0;
    while (next < n) {
        Slot& s = ctx->slot[k % kSlots];
        int rc = drain(s);
        if (rc) return rc;
        uint64_t used = 0;
        uint32_t cnt = 0;
        const uint8_t* h2d_src = s.h_frames;
        // span mode: frames in place in the caller's pinned buffer
        if (pinned && (off[next] & 15) == 0) {
            const uint64_t s0 = off[next];
            uint64_t prev = s0;
            while (next + cnt < n && cnt < ctx->max_frames) {
                uint32_t i = next + cnt;
                if ((off[i] & 15) || off[i] < prev || off[i] + len[i] - s0 > ctx->max_bytes)
                    break;
                s.h_off[cnt] = off[i] - s0;
                s.h_len[cnt] = len[i];
                used = std::max<uint64_t>(used, off[i] + len[i] - s0);
                prev = off[i];
                cnt++;
            }
            h2d_src = base + s0;
        }
        // gather mode
        uint8_t* gdst = s.h_frames;
        if (cnt == 0) {
            h2d_src = s.h_frames;
            while (next + cnt < n && cnt < ctx->max_frames) {
                uint32_t i = next + cnt;
                uint64_t need = (len[i] + kSlotAlign - 1) / kSlotAlign * kSlotAlign;
                if (used + need > ctx->max_bytes)
                    break;
                s.h_off[cnt] = used;
                s.h_len[cnt] = frame_ptr(i) ? len[i] : 0;
                used += need;
                cnt++;
            }
            if (cnt == 0)
                return GCS_ERANGE;   // a single frame larger than the staging
            if (ctx->direct_stage_dev && next == 0 && cnt == n && used <= ctx->direct_max) {
                // a gathered batch never exceeds the slot's pinned staging
                if (!s.v_frames &&
                    hipExtMallocWithFlags((void**)&s.v_frames,
                                          std::min(ctx->direct_max, ctx->max_bytes),
                                          hipDeviceMallocFinegrained) != hipSuccess) {
                    (void)hipGetLastError();
                    s.v_frames = nullptr;
                    ctx->direct_stage_dev = false;      // no host-mapped device memory
                }
                if (s.v_frames)
                    gdst = s.v_frames;
            }
            const uint32_t first = next;
            ctx->gather_run(cnt, used, [&, first](uint32_t lo, uint32_t hi) {
                for (uint32_t k = lo; k < hi; k++) {
                    const uint8_t* src = frame_ptr(first + k);
                    if (src)
                        std::memcpy(gdst + s.h_off[k], src, s.h_len[k]);
                }
            });
            // device staging is written over the BAR, write-combined: drain
            // it before the request's seq publishes the batch
            if (gdst != s.h_frames)
                __builtin_ia32_sfence();
        }
        s.first = next;
        s.count = cnt;
        // Direct mode: a small batch staged whole in one gather (an mTCP burst is
        // <= 64 frames, dpdk_module.c:76).  The kernel reads the pinned staging
        // and writes its results over PCIe: one launch instead of three H2D
        // copies + the kernel + one or three D2H copies, each with its own
        // submission latency.
        const bool direct = h2d_src == s.h_frames && next == 0 && cnt == n &&
                            used <= ctx->direct_max;
        uint8_t* frames_d = direct ? (gdst != s.h_frames ? s.v_frames : s.m_frames) : s.d_frames;
        uint64_t* off_d = direct ? s.m_off : s.d_off;
        uint16_t* len_d = direct ? s.m_len : s.d_len;
        uint8_t* code_d = direct ? s.m_code : s.d_code;
        uint32_t* csum_d = direct ? s.m_csum : s.d_csum;
        uint32_t* hash_d = direct ? s.m_hash : s.d_hash;
        uint16_t* queue_d = direct ? s.m_queue : s.d_queue;
        if (!direct) {
            HIP_TRY(hipMemcpyAsync(s.d_frames, h2d_src, used, hipMemcpyHostToDevice, s.stream));
            HIP_TRY(hipMemcpyAsync(s.d_off, s.h_off, cnt * sizeof(uint64_t),
                                   hipMemcpyHostToDevice, s.stream));
            HIP_TRY(hipMemcpyAsync(s.d_len, s.h_len, cnt * sizeof(uint16_t),
                                   hipMemcpyHostToDevice, s.stream));
        }
        const bool spread = direct && ctx->direct_spread && !(flags & GCS_VF_ICMP);
        if (spread && !classify && ctx->server && cnt <= (uint32_t)gcs::kServerMaxFrames) {
            // resident grid: no launch, no event; results complete on return
            int rc = ctx->server->serve(frames_d, (used + 15) / 16 * 16, s.h_off, s.h_len, cnt,
                                        compute, compute ? GCS_CF_NO_INPLACE : 0u, s.h_code,
                                        compute ? s.h_csum : nullptr, false,
                                        gdst != s.h_frames ? gcs::kModeDevFrames : 0u);
            if (rc) return rc;
            s.busy = true;
            s.served = true;
            next += cnt;
            k++;
            continue;
        }
        if (ctx->server) {
            // other work on this context's streams: its posted requests
            // complete first, in order
            int rc = ctx->server->stop();
            if (rc) return rc;
        }
        if (spread && !classify) {
            // direct mode: the results come back as whole 64 B lines of
            // records (k_desc_rec), unpacked by drain()
            HIP_TRY(gcs::launch_desc_rec(frames_d, used, off_d, len_d, cnt, s.m_rec, compute,
                                         compute ? (uint32_t)GCS_CF_NO_INPLACE : 0u, s.stream));
            s.rec = true;
        } else if (compute) {
            HIP_TRY(gcs::launch_compute_desc(frames_d, used, off_d, len_d, cnt, code_d, csum_d,
                                             GCS_CF_NO_INPLACE, s.stream));
            if (!direct)
                HIP_TRY(hipMemcpyAsync(s.h_csum, s.d_csum, cnt * sizeof(uint32_t),
                                       hipMemcpyDeviceToHost, s.stream));
        } else if (classify) {
            HIP_TRY(gcs::launch_classify_desc(frames_d, used, off_d, len_d, cnt, code_d,
                                              flags & GCS_VF_ICMP,
                                              rss_ext(ctx, hash_d, queue_d), s.stream));
            if (hash && !direct)
                HIP_TRY(hipMemcpyAsync(s.h_hash, s.d_hash, cnt * sizeof(uint32_t),
                                       hipMemcpyDeviceToHost, s.stream));
            if (queue && !direct)
                HIP_TRY(hipMemcpyAsync(s.h_queue, s.d_queue, cnt * sizeof(uint16_t),
                                       hipMemcpyDeviceToHost, s.stream));
        } else {
            // the tcp_in.c:1237 side effect is applied on the host copy below
            HIP_TRY(gcs::launch_verify_desc(frames_d, used, off_d, len_d, cnt, code_d,
                                            flags & GCS_VF_ICMP, s.stream));
        }
        if (!direct)
            HIP_TRY(hipMemcpyAsync(s.h_code, s.d_code, cnt, hipMemcpyDeviceToHost, s.stream));
        HIP_TRY(hipEventRecord(s.done, s.stream));
        s.busy = true;
        next += cnt;
        k++;
        if (k == 1 && next < n && fault("second_chunk"))   // a HIP failure mid-batch
            return hip_fail(hipErrorLaunchFailure, "injected before chunk 2");
    }
    for (auto& s : ctx->slot) {
        int rc = drain(s);
        if (rc) return rc;
    }
    if (!compute && (flags & GCS_VF_ZERO_BAD_TCP_CHECK))
        zero_bad_tcp_checks(code, n, frame_ptr, len);
    return GCS_OK;
}

}  // namespace

extern "C" {

int gcs_abi_version(void) { return GCS_ABI_VERSION; }

const char* gcs_strerror(int code)
{
    switch (code) {
    case GCS_OK: return "ok";
    case GCS_EINVAL: return "invalid argument";
    case GCS_ENODEV: return "no such HIP device";
    case GCS_ENOMEM: return "out of memory";
    case GCS_EHIP: return "HIP runtime error";
    case GCS_ERANGE: return "batch exceeds context capacity";
    default: return "unknown error";
    }
}

const char* gcs_last_hip_error(void) { return g_hip_err; }

int gcs_device_count(int* count)
try {
    if (!count)
        return GCS_EINVAL;
    int c = 0;
    hipError_t e = hipGetDeviceCount(&c);
    if (e != hipSuccess) {
        *count = 0;
        return hip_fail(e, "hipGetDeviceCount");
    }
    *count = c;
    return GCS_OK;
} GCS_CATCH

int gcs_ctx_create(gcs_ctx** out, int device, uint32_t max_frames, uint64_t max_bytes)
try {
    if (!out)
        return GCS_EINVAL;
    *out = nullptr;
    int count = 0;
    int rc = gcs_device_count(&count);
    if (rc)
        return rc;
    if (device < 0 || device >= count)
        return GCS_ENODEV;
    gcs_ctx* ctx = new (std::nothrow) gcs_ctx();
    if (!ctx)
        return GCS_ENOMEM;
    ctx->device = device;
    DeviceGuard g(device);
    hipError_t e = hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking);
    if (e != hipSuccess) {
        delete ctx;
        return hip_fail(e, "hipStreamCreateWithFlags");
    }
    set_rss_params(ctx, kDefaultRssKey, 1, 0);
    ctx->direct_max = kDirectMaxBytes;
    if (const char* e = std::getenv("GCS_DIRECT_MAX_BYTES"))
        ctx->direct_max = std::strtoull(e, nullptr, 10);
    if (const char* e = std::getenv("GCS_DIRECT_SPREAD"))
        ctx->direct_spread = std::atoi(e) != 0;
    if (const char* e = std::getenv("GCS_ASYNC_STAGE"))
        ctx->async_stage_dev = std::strcmp(e, "host") != 0;
    if (const char* e = std::getenv("GCS_DIRECT_STAGE"))
        ctx->direct_stage_dev = std::strcmp(e, "host") != 0;
    if (const char* e = std::getenv("GCS_ASYNC_REGISTERED"))
        ctx->async_reg_stage = std::strcmp(e, "inplace") != 0;
    ctx->faults = std::getenv("GCS_FAULT_INJECT") != nullptr;
    if (const char* e = std::getenv("GCS_BURST_SERVER")) {
        // a context beyond the grid's kHubRings runs without it (GCS_ERANGE)
        if (std::atoi(e) != 0 && (rc = gcs_ctx_set_burst_server(ctx, 1)) != GCS_OK &&
            rc != GCS_ERANGE) {
            gcs_ctx_destroy(ctx);
            return rc;
        }
    }
    if (max_frames && max_bytes) {
        // split the requested staging between the two slots
        ctx->max_frames = std::max<uint32_t>(1, max_frames / kSlots + 1);
        ctx->max_bytes = (max_bytes / kSlots + kSlotAlign + 2047) / kSlotAlign * kSlotAlign;
        for (auto& s : ctx->slot) {
            rc = alloc_slot(s, ctx->max_frames, ctx->max_bytes);
            if (rc) {
                gcs_ctx_destroy(ctx);
                return rc;
            }
        }
    }
    *out = ctx;
    return GCS_OK;
} GCS_CATCH

// Everything is released whatever fails; the first failure is returned (a
// device fault surfacing at teardown is this context's, not the next
// caller's).  The ring leaves the grid before any staging it served is freed.
int gcs_ctx_destroy(gcs_ctx* ctx)
try {
    if (!ctx)
        return GCS_EINVAL;
    int rc = GCS_OK;
    {
        DeviceGuard g(ctx->device);
        if (ctx->server) {
            rc = ctx->server->shutdown();   // its requests complete; the ring leaves the grid
            ctx->server.reset();
        }
        for (auto& a : ctx->areq)
            if (a.h_stage)
                keep_first(rc, a.stage_dev ? hipFree(a.h_stage) : hipHostFree(a.h_stage),
                           "async staging free");
        for (auto& s : ctx->slot) {
            const int e = free_slot(s);
            if (rc == GCS_OK) rc = e;
        }
        if (ctx->stream) {
            keep_first(rc, hipStreamSynchronize(ctx->stream), "context stream sync");
            keep_first(rc, hipStreamDestroy(ctx->stream), "hipStreamDestroy");
        }
    }
    delete ctx;
    return rc;
} GCS_CATCH

int gcs_device_check(int device)
try {
    int count = 0;
    int rc = gcs_device_count(&count);
    if (rc)
        return rc;
    if (device < 0 || device >= count)
        return GCS_ENODEV;
    DeviceGuard g(device);
    if (ServerHub* h = ServerHub::peek(device)) {
        rc = h->check_idle();
        if (rc)
            return rc;
    }
    HIP_TRY(hipDeviceSynchronize());
    // a fault is reported to the process asynchronously (its interrupt is
    // handled after the faulting kernel may have completed): look again
    // after a moment, so it is charged to the work that caused it
    std::this_thread::sleep_for(std::chrono::milliseconds(1));
    HIP_TRY(hipDeviceSynchronize());
    return GCS_OK;
} GCS_CATCH

int gcs_ctx_device(const gcs_ctx* ctx, int* device)
try {
    if (!ctx || !device)
        return GCS_EINVAL;
    *device = ctx->device;
    return GCS_OK;
} GCS_CATCH

int gcs_ctx_stream(const gcs_ctx* ctx, void** stream)
try {
    if (!ctx || !stream)
        return GCS_EINVAL;
    *stream = ctx->stream;
    return GCS_OK;
} GCS_CATCH

int gcs_sync(gcs_ctx* ctx)
try {
    if (!ctx)
        return GCS_EINVAL;
    DeviceGuard g(ctx->device);
    HIP_TRY(hipStreamSynchronize(ctx->stream));
    return GCS_OK;
} GCS_CATCH

int gcs_host_alloc(void** p, uint64_t bytes)
try {
    if (!p)
        return GCS_EINVAL;
    HIP_TRY(hipHostMalloc(p, bytes, hipHostMallocDefault));
    return GCS_OK;
} GCS_CATCH

int gcs_host_free(void* p)
try {
    HIP_TRY(hipHostFree(p));
    return GCS_OK;
} GCS_CATCH

// Regions are process-wide.  The burst server's request carries a region's
// size in 16 B units as a u32, hence the 64 GiB limit.  hipHostRegister maps
// the pages for every device of the process (one address space), so the
// device view is valid whichever device the calling thread has current.
int gcs_host_register(void* p, uint64_t bytes)
try {
    if (!p || bytes == 0 || bytes / 16 > 0xFFFFFFFFull)
        return GCS_EINVAL;
    uint8_t* const host = static_cast<uint8_t*>(p);
    std::lock_guard<std::mutex> lk(g_reg_mu);
    for (const auto& r : g_regions)
        if (host < r.host + r.bytes && r.host < host + bytes)
            return GCS_EINVAL;                        // overlaps a registered region
    // Uncached (MTYPE UC) by default: the burst server then reads a region's
    // frames without invalidating the L2 first (the acquire after each poll,
    // ~1 us per RX burst); GCS_REGISTER_UNCACHED=0, or a runtime without the
    // flag, registers it cached (then every request takes the acquire).
    const char* uc = std::getenv("GCS_REGISTER_UNCACHED");
    bool uncached = !uc || std::strcmp(uc, "0") != 0;
    if (uncached &&
        hipHostRegister(p, bytes, hipHostRegisterMapped | hipExtHostRegisterUncached) !=
            hipSuccess) {
        (void)hipGetLastError();
        uncached = false;
    }
    if (!uncached)
        HIP_TRY(hipHostRegister(p, bytes, hipHostRegisterMapped));
    uint8_t* dev = nullptr;
    hipError_t e = hipHostGetDevicePointer((void**)&dev, p, 0);
    if (e != hipSuccess) {
        (void)hipHostUnregister(p);
        return hip_fail(e, "hipHostGetDevicePointer");
    }
    g_regions.push_back(RegRegion{host, bytes, dev, uncached});
    return GCS_OK;
} GCS_CATCH

int gcs_host_unregister(void* p)
try {
    if (!p)
        return GCS_EINVAL;
    {
        std::lock_guard<std::mutex> lk(g_reg_mu);
        for (auto it = g_regions.begin(); it != g_regions.end(); ++it)
            if (it->host == p) {
                g_regions.erase(it);
                break;
            }
    }
    HIP_TRY(hipHostUnregister(p));
    return GCS_OK;
} GCS_CATCH

int gcs_dev_alloc(gcs_ctx* ctx, void** p, uint64_t bytes)
try {
    if (!ctx || !p)
        return GCS_EINVAL;
    DeviceGuard g(ctx->device);
    HIP_TRY(hipMalloc(p, bytes));
    return GCS_OK;
} GCS_CATCH

int gcs_dev_free(gcs_ctx* ctx, void* p)
try {
    if (!ctx)
        return GCS_EINVAL;
    DeviceGuard g(ctx->device);
    HIP_TRY(hipFree(p));
    return GCS_OK;
} GCS_CATCH

int gcs_verify_fixed_dev(gcs_ctx* ctx, uint8_t* d_frames, uint64_t stride, uint32_t frame_len,
                         uint32_t n, uint8_t* d_verdict, uint32_t flags, void* stream)
try {
    if (!ctx || (n && (!d_frames || !d_verdict)) || stride % 16 || stride == 0 ||
        (frame_len + 15u) / 16u * 16u > stride)
        return GCS_EINVAL;
    if (n == 0)
        return GCS_OK;
    DeviceGuard g(ctx->device);
    HIP_TRY(gcs::launch_verify_fixed(d_frames, stride, frame_len, n, d_verdict, flags,
                                     pick_stream(ctx, stream)));
    return GCS_OK;
} GCS_CATCH

int gcs_compute_fixed_dev(gcs_ctx* ctx, uint8_t* d_frames, uint64_t stride, uint32_t frame_len,
                          uint32_t n, uint8_t* d_status, uint32_t* d_csums, uint32_t flags,
                          void* stream)
try {
    if (!ctx || (n && !d_frames) || stride % 16 || stride == 0 ||
        (frame_len + 15u) / 16u * 16u > stride)
        return GCS_EINVAL;
    if (n == 0)
        return GCS_OK;
    DeviceGuard g(ctx->device);
    HIP_TRY(gcs::launch_compute_fixed(d_frames, stride, frame_len, n, d_status, d_csums, flags,
                                      pick_stream(ctx, stream)));
    return GCS_OK;
} GCS_CATCH

int gcs_step_fixed_dev(gcs_ctx* ctx, uint8_t* d_tx, uint64_t tx_stride, uint32_t tx_len,
                       uint32_t n_tx, uint8_t* d_tx_status, uint32_t* d_tx_csums,
                       uint32_t tx_flags, uint8_t* d_rx, uint64_t rx_stride, uint32_t rx_len,
                       uint32_t n_rx, uint8_t* d_rx_verdict, uint32_t rx_flags, void* stream)
try {
    auto bad_shape = [](uint64_t stride, uint32_t len) {
        return stride % 16 || stride == 0 || (len + 15u) / 16u * 16u > stride;
    };
    if (!ctx || (n_tx && (!d_tx || bad_shape(tx_stride, tx_len))) ||
        (n_rx && (!d_rx || !d_rx_verdict || bad_shape(rx_stride, rx_len))))
        return GCS_EINVAL;
    if (n_tx && n_rx) {
        // the one launch runs both at once: they may not share a byte
        const uint64_t t0 = reinterpret_cast<uint64_t>(d_tx), t1 = t0 + (uint64_t)n_tx * tx_stride;
        const uint64_t r0 = reinterpret_cast<uint64_t>(d_rx), r1 = r0 + (uint64_t)n_rx * rx_stride;
        if (t0 < r1 && r0 < t1)
            return GCS_EINVAL;
    }
    if (n_tx == 0 && n_rx == 0)
        return GCS_OK;
    DeviceGuard g(ctx->device);
    HIP_TRY(gcs::launch_step_fixed(d_tx, tx_stride, tx_len, n_tx, d_tx_status, d_tx_csums,
                                   tx_flags, d_rx, rx_stride, rx_len, n_rx, d_rx_verdict, rx_flags,
                                   pick_stream(ctx, stream)));
    return GCS_OK;
} GCS_CATCH

int gcs_verify_dev(gcs_ctx* ctx, uint8_t* d_frames, uint64_t frames_bytes, const uint64_t* d_off,
                   const uint16_t* d_len, uint32_t n, uint8_t* d_verdict, uint32_t flags,
                   void* stream)
try {
    if (!ctx || (n && (!d_frames || !d_off || !d_len || !d_verdict)))
        return GCS_EINVAL;
    if (n == 0)
        return GCS_OK;
    DeviceGuard g(ctx->device);
    const hipStream_t st = pick_stream(ctx, stream);
    HIP_TRY(gcs::launch_verify_desc(d_frames, frames_bytes, d_off, d_len, n, d_verdict, flags, st));
    return GCS_OK;
} GCS_CATCH

int gcs_compute_dev(gcs_ctx* ctx, uint8_t* d_frames, uint64_t frames_bytes, const uint64_t* d_off,
                    const uint16_t* d_len, uint32_t n, uint8_t* d_status, uint32_t* d_csums,
                    uint32_t flags, void* stream)
try {
    if (!ctx || (n && (!d_frames || !d_off || !d_len)))
        return GCS_EINVAL;
    if (n == 0)
        return GCS_OK;
    DeviceGuard g(ctx->device);
    const hipStream_t st = pick_stream(ctx, stream);
    HIP_TRY(gcs::launch_compute_desc(d_frames, frames_bytes, d_off, d_len, n, d_status, d_csums,
                                     flags, st));
    return GCS_OK;
} GCS_CATCH

int gcs_tcp_checksum_dev(gcs_ctx* ctx, const uint8_t* d_buf, uint64_t buf_bytes,
                         const uint64_t* d_off, const uint16_t* d_len, const uint32_t* d_saddr,
                         const uint32_t* d_daddr, uint32_t n, uint16_t* d_out, void* stream)
try {
    if (!ctx || (n && (!d_buf || !d_off || !d_len || !d_saddr || !d_daddr || !d_out)))
        return GCS_EINVAL;
    if (n == 0)
        return GCS_OK;
    DeviceGuard g(ctx->device);
    HIP_TRY(gcs::launch_tcp_fn(d_buf, buf_bytes, d_off, d_len, d_saddr, d_daddr, n, d_out,
                               pick_stream(ctx, stream)));
    return GCS_OK;
} GCS_CATCH

int gcs_ip_checksum_dev(gcs_ctx* ctx, const uint8_t* d_buf, uint64_t buf_bytes,
                        const uint64_t* d_off, const uint8_t* d_ihl, uint32_t n, uint16_t* d_out,
                        void* stream)
try {
    if (!ctx || (n && (!d_buf || !d_off || !d_ihl || !d_out)))
        return GCS_EINVAL;
    if (n == 0)
        return GCS_OK;
    DeviceGuard g(ctx->device);
    HIP_TRY(gcs::launch_ip_fn(d_buf, buf_bytes, d_off, d_ihl, n, d_out, pick_stream(ctx, stream)));
    return GCS_OK;
} GCS_CATCH

int gcs_compute_copy_dev(gcs_ctx* ctx, uint8_t* d_frames, uint64_t frames_bytes,
                         const uint64_t* d_off, const uint16_t* d_len, const uint8_t* d_src,
                         uint64_t src_bytes, const uint64_t* d_src_off, uint32_t n,
                         uint8_t* d_status, uint32_t* d_csums, uint32_t flags, void* stream)
try {
    if (!ctx || flags != 0 || (n && (!d_frames || !d_off || !d_len || !d_src || !d_src_off)))
        return GCS_EINVAL;
    if (n == 0)
        return GCS_OK;
    DeviceGuard g(ctx->device);
    HIP_TRY(gcs::launch_copy_fill(d_frames, frames_bytes, d_off, d_len, d_src, src_bytes,
                                  d_src_off, n, d_status, d_csums, flags,
                                  pick_stream(ctx, stream)));
    return GCS_OK;
} GCS_CATCH

int gcs_gro_dev(gcs_ctx* ctx, const uint8_t* d_in, uint64_t in_bytes, const uint64_t* d_off,
                const uint16_t* d_len, const uint8_t* d_verdict, uint32_t n, uint32_t window,
                uint32_t max_len, uint8_t* d_out, uint64_t out_bytes, uint64_t* d_out_off,
                uint16_t* d_out_len, uint32_t* d_head, void* stream)
try {
    if (!ctx || window == 0 || window > 256 || max_len > 65535 ||
        (n && (!d_in || !d_off || !d_len || !d_verdict || !d_out || !d_out_off || !d_out_len ||
               !d_head)))
        return GCS_EINVAL;
    if (n == 0)
        return GCS_OK;
    DeviceGuard g(ctx->device);
    HIP_TRY(gcs::launch_gro(d_in, in_bytes, d_off, d_len, d_verdict, n, window, max_len, d_out,
                            out_bytes, d_out_off, d_out_len, d_head, pick_stream(ctx, stream)));
    return GCS_OK;
} GCS_CATCH

int gcs_icmp_checksum_dev(gcs_ctx* ctx, const uint8_t* d_buf, uint64_t buf_bytes,
                          const uint64_t* d_off, const uint16_t* d_len, uint32_t n,
                          uint16_t* d_out, void* stream)
try {
    if (!ctx || (n && (!d_buf || !d_off || !d_len || !d_out)))
        return GCS_EINVAL;
    if (n == 0)
        return GCS_OK;
    DeviceGuard g(ctx->device);
    HIP_TRY(gcs::launch_icmp_fn(d_buf, buf_bytes, d_off, d_len, n, d_out,
                                pick_stream(ctx, stream)));
    return GCS_OK;
} GCS_CATCH

int gcs_ctx_set_burst_server(gcs_ctx* ctx, int on)
try {
    if (!ctx)
        return GCS_EINVAL;
    DeviceGuard g(ctx->device);
    if (!on) {
        const int rc = ctx->server ? ctx->server->shutdown() : GCS_OK;
        ctx->server.reset();
        return rc;
    }
    if (ctx->server)
        return GCS_OK;
    std::unique_ptr<BurstServer> sv(new BurstServer());
    int rc = sv->init(ctx->device);
    if (rc)
        return rc;
    ctx->server = std::move(sv);
    return GCS_OK;
} GCS_CATCH

int gcs_server_stats_get(gcs_ctx* ctx, gcs_server_stats* out)
try {
    if (!ctx || !out || !ctx->server)
        return GCS_EINVAL;
    ctx->server->stats(out);
    return GCS_OK;
} GCS_CATCH

int gcs_ctx_set_rss(gcs_ctx* ctx, const uint8_t* key, uint32_t key_len, uint32_t num_queues,
                    int endian_check)
try {
    if (!ctx || num_queues == 0 || num_queues > 0xFFFFu || (key && key_len < 16))
        return GCS_EINVAL;
    uint8_t k[40];
    std::memcpy(k, kDefaultRssKey, sizeof k);
    if (key)
        std::memcpy(k, key, std::min<uint32_t>(key_len, sizeof k));
    // the parameters travel by value in each launch: no device state to fence
    set_rss_params(ctx, k, num_queues, endian_check ? 1u : 0u);
    return GCS_OK;
} GCS_CATCH

int gcs_classify_fixed_dev(gcs_ctx* ctx, uint8_t* d_frames, uint64_t stride, uint32_t frame_len,
                           uint32_t n, uint8_t* d_verdict, uint32_t* d_hash, uint16_t* d_queue,
                           uint32_t flags, void* stream)
try {
    if (!ctx || (n && (!d_frames || !d_verdict)) || stride % 16 || stride == 0 ||
        (frame_len + 15u) / 16u * 16u > stride)
        return GCS_EINVAL;
    if (n == 0)
        return GCS_OK;
    DeviceGuard g(ctx->device);
    HIP_TRY(gcs::launch_classify_fixed(d_frames, stride, frame_len, n, d_verdict, flags,
                                       rss_ext(ctx, d_hash, d_queue), pick_stream(ctx, stream)));
    return GCS_OK;
} GCS_CATCH

int gcs_classify_dev(gcs_ctx* ctx, uint8_t* d_frames, uint64_t frames_bytes,
                     const uint64_t* d_off, const uint16_t* d_len, uint32_t n,
                     uint8_t* d_verdict, uint32_t* d_hash, uint16_t* d_queue, uint32_t flags,
                     void* stream)
try {
    if (!ctx || (n && (!d_frames || !d_off || !d_len || !d_verdict)))
        return GCS_EINVAL;
    if (n == 0)
        return GCS_OK;
    DeviceGuard g(ctx->device);
    HIP_TRY(gcs::launch_classify_desc(d_frames, frames_bytes, d_off, d_len, n, d_verdict, flags,
                                      rss_ext(ctx, d_hash, d_queue), pick_stream(ctx, stream)));
    return GCS_OK;
} GCS_CATCH

int gcs_rss_dev(gcs_ctx* ctx, const uint32_t* d_sip, const uint32_t* d_dip, const uint16_t* d_sp,
                const uint16_t* d_dp, uint32_t n, uint32_t* d_hash, uint16_t* d_queue,
                void* stream)
try {
    if (!ctx || (n && (!d_sip || !d_dip || !d_sp || !d_dp || (!d_hash && !d_queue))))
        return GCS_EINVAL;
    if (n == 0)
        return GCS_OK;
    DeviceGuard g(ctx->device);
    HIP_TRY(gcs::launch_rss_fn(d_sip, d_dip, d_sp, d_dp, n, rss_ext(ctx, d_hash, d_queue),
                               pick_stream(ctx, stream)));
    return GCS_OK;
} GCS_CATCH

int gcs_classify(gcs_ctx* ctx, uint8_t* frames, const uint64_t* off, const uint16_t* len,
                 uint32_t n, uint8_t* verdict, uint32_t* hash, uint16_t* queue, uint32_t flags)
try {
    if (!hash && !queue)
        return GCS_EINVAL;
    return run_host_batch(ctx, frames, off, nullptr, len, n, verdict, nullptr, flags, false,
                          hash, queue);
} GCS_CATCH

int gcs_classify_ptrs(gcs_ctx* ctx, uint8_t* const* pkts, const uint16_t* len, uint32_t n,
                      uint8_t* verdict, uint32_t* hash, uint16_t* queue, uint32_t flags)
try {
    if (!hash && !queue)
        return GCS_EINVAL;
    if (ctx && ctx->faults && n && fault("verify_ptrs"))   // test-only (plugin RX failure)
        return hip_fail(hipErrorLaunchFailure, "injected (verify_ptrs)");
    return run_host_batch(ctx, nullptr, nullptr, pkts, len, n, verdict, nullptr, flags, false,
                          hash, queue);
} GCS_CATCH

int gcs_verify(gcs_ctx* ctx, uint8_t* frames, const uint64_t* off, const uint16_t* len,
               uint32_t n, uint8_t* verdict, uint32_t flags)
try {
    return run_host_batch(ctx, frames, off, nullptr, len, n, verdict, nullptr, flags, false);
} GCS_CATCH

int gcs_compute(gcs_ctx* ctx, uint8_t* frames, const uint64_t* off, const uint16_t* len,
                uint32_t n, uint8_t* status, uint32_t* csums)
try {
    return run_host_batch(ctx, frames, off, nullptr, len, n, status, csums, 0u, true);
} GCS_CATCH

namespace {

constexpr uint64_t kAsyncStageBytes = 256u << 10;   // per server slot

// Finish async request a: its server request is done (results in a.st /
// a.cs).  A fill: the caller's statuses / checks and the frames' check fields.
// A verify: the caller's verdicts, and the tcp_in.c:1237 side effect
// (GCS_VF_ZERO_BAD_TCP_CHECK) on the frames themselves.
void async_finish(gcs_ctx::AsyncReq& a)
{
    if (!a.compute) {
        if (a.status)
            std::memcpy(a.status, a.st.data(), a.n);
        if (a.flags & GCS_VF_ZERO_BAD_TCP_CHECK)
            zero_bad_tcp_checks(a.st.data(), a.n,
                                [&](uint32_t i) -> uint8_t* { return a.ptrs[i]; }, a.lens.data());
        a.pending = false;
        return;
    }
    for (uint32_t i = 0; i < a.n; i++) {
        if (a.status) a.status[i] = a.st[i];
        if (a.csums) a.csums[i] = a.cs[i];
        if (a.ptrs[i])
            scatter_tx(a.ptrs[i], a.lens[i], a.st[i], a.cs[i]);
    }
    a.pending = false;
}

// The kind of async request q (1: fill, 0: verify), or -1 when its slot no
// longer holds it.
int ticket_kind(const gcs_ctx* ctx, uint32_t q)
{
    const gcs_ctx::AsyncReq& a = ctx->areq[q % gcs::kServerSlots];
    return a.q == q ? (a.compute ? 1 : 0) : -1;
}

// report = false: a post draining its slot's previous request, which leaves
// the loss of cancelled requests to their own waiters.
int async_wait(gcs_ctx* ctx, uint32_t q, bool report = true)
{
    DeviceGuard g(ctx->device);
    if (ctx->server) {
        // test-only GCS_FAULT_INJECT=wait: the server "gives no answer"
        int rc = ctx->faults && fault("wait") ? hip_fail(hipErrorLaunchFailure, "injected (wait)")
                               : ctx->server->wait(q);
        if (rc) {
            // The server did not answer: cancel every pending async request,
            // so that no later wait writes an old request's checks into
            // buffers the caller has since reused (the caller treats the
            // frames as unfilled / unverified; the library forgets their
            // addresses here).  The staging slot itself is reused only after
            // its server request completes (BurstServer::post waits for it
            // first).  This failure is the report for every cancelled request
            // of the waiter's kind up to the ticket it waited for; any other
            // cancelled request -- a later one of its kind, or one of the
            // other kind -- is reported once, to the first later wait of its
            // kind that covers it (a wait for its own ticket included: it
            // never reads as done).
            const int kind = ticket_kind(ctx, q);
            for (auto& a : ctx->areq) {
                const bool reported = (kind < 0 || kind == a.compute) &&
                                      (int32_t)(q - a.q) >= 0;
                if (a.pending) {
                    a.pending = false;
                    a.cancelled = !reported;
                    std::fill(a.ptrs.begin(), a.ptrs.end(), nullptr);
                    a.status = nullptr;
                    a.csums = nullptr;
                } else if (reported) {
                    a.cancelled = false;        // reported by this failure
                }
            }
            return rc;
        }
    }
    // A request a failed wait cancelled is "lost" for the first later wait
    // that covers it and waits for a request of the same kind (fills and
    // verifies share the ring; the plugin's TX and RX paths each wait for
    // their own tickets): it is reported once and forgotten, so requests
    // posted after the failure that the server completed are never reported.
    const int kind = ticket_kind(ctx, q);
    bool lost = false;
    for (auto& a : ctx->areq) {
        if (report && a.cancelled && (int32_t)(q - a.q) >= 0 &&
            (kind < 0 || kind == a.compute)) {
            lost = true;
            a.cancelled = false;
        }
        if (a.pending && (int32_t)(q - a.q) >= 0)
            async_finish(a);
    }
    if (lost) {
        std::snprintf(g_hip_err, sizeof g_hip_err,
                      "async request cancelled by an earlier failed wait");
        return GCS_EHIP;
    }
    return GCS_OK;
}

}  // namespace

namespace {

// One async request on the context's burst server: a TX fill (compute) or an
// RX verify.  Frames all in one registered region at 16 B-aligned addresses
// are read where they are; others are staged in the request slot's pinned
// (or, GCS_ASYNC_STAGE=device, device) staging.  *ticket = 0 when the batch
// could not be posted and ran synchronously instead.
int post_async(gcs_ctx* ctx, uint8_t* const* pkts, const uint16_t* len, uint32_t n, bool compute,
               uint32_t flags, uint8_t* out8, uint32_t* csums, uint64_t* ticket)
{
    auto sync = [&]() {
        return compute ? run_host_batch(ctx, nullptr, nullptr, pkts, len, n, out8, csums, 0u, true)
                       : run_host_batch(ctx, nullptr, nullptr, pkts, len, n, out8, nullptr, flags,
                                        false);
    };
    if (!ctx->server || n > (uint32_t)gcs::kSlotFrames ||
        (!compute && (flags & ~(uint32_t)GCS_VF_ZERO_BAD_TCP_CHECK)))
        return sync();
    DeviceGuard g(ctx->device);
    // in place: every frame inside one registered region, 16 B-aligned
    RegRegion reg{};
    uint32_t first = 0;
    while (first < n && !pkts[first])
        first++;
    bool inplace = first < n && !(ctx->async_reg_stage && ctx->async_stage_dev) &&
                   find_region(pkts[first], &reg);
    uint64_t staged = 0;
    for (uint32_t i = 0; i < n; i++) {
        staged += (len[i] + kSlotAlign - 1) / kSlotAlign * kSlotAlign;
        const uint8_t* p = pkts[i];
        if (inplace && p)
            inplace = p >= reg.host && (uint64_t)(p - reg.host) + len[i] <= (reg.bytes & ~15ull) &&
                      ((uintptr_t)p & 15) == 0;
    }
    if (!inplace && staged > kAsyncStageBytes)
        return sync();
    const uint32_t q = gcs::server_next(ctx->server->posted());
    gcs_ctx::AsyncReq& a = ctx->areq[q % gcs::kServerSlots];
    if (a.pending) {                     // the slot's previous async request: finish it first
        int rc = async_wait(ctx, a.q, /*report=*/false);
        if (rc) return rc;
    }
    a.cancelled = false;                 // nobody waited for that one: the slot is reused
    if (a.st.size() < (size_t)gcs::kSlotFrames) {
        a.ptrs.resize(gcs::kSlotFrames);
        a.lens.resize(gcs::kSlotFrames);
        a.off.resize(gcs::kSlotFrames);
        a.dlen.resize(gcs::kSlotFrames);
        a.st.resize(gcs::kSlotFrames);
        a.cs.resize(gcs::kSlotFrames);
    }
    a.staged = !inplace;
    uint8_t* frames_d = reg.dev;
    uint64_t bytes = reg.bytes & ~15ull;
    if (a.staged) {
        if (!a.h_stage) {
            if (ctx->async_stage_dev &&
                hipExtMallocWithFlags((void**)&a.h_stage, kAsyncStageBytes,
                                      hipDeviceMallocFinegrained) != hipSuccess) {
                (void)hipGetLastError();
                a.h_stage = nullptr;
                ctx->async_stage_dev = false;           // no host-mapped device memory
            }
            if (a.h_stage) {
                // staging in fine-grained device memory, written by the host
                // over the BAR: the GPU then reads the frames from HBM
                a.d_stage = a.h_stage;
                a.stage_dev = true;
            } else {
                HIP_TRY(hipHostMalloc((void**)&a.h_stage, kAsyncStageBytes,
                                      hipHostMallocDefault));
                HIP_TRY(hipHostGetDevicePointer((void**)&a.d_stage, a.h_stage, 0));
            }
        }
        uint64_t used = 0;
        for (uint32_t i = 0; i < n; i++) {
            a.off[i] = used;
            a.dlen[i] = pkts[i] ? len[i] : 0;
            if (pkts[i])
                std::memcpy(a.h_stage + used, pkts[i], len[i]);
            used += (len[i] + kSlotAlign - 1) / kSlotAlign * kSlotAlign;
        }
        // Device staging is mapped write-combining over the BAR: drain the WC
        // buffers before post() publishes seq (a release store is a plain mov
        // on x86 and orders nothing against WC stores), so the server never
        // sees the request before its frame bytes.
        if (a.stage_dev)
            __builtin_ia32_sfence();
        frames_d = a.d_stage;
        bytes = (used + 15) / 16 * 16;
    } else {
        for (uint32_t i = 0; i < n; i++) {
            a.off[i] = pkts[i] ? (uint64_t)(pkts[i] - reg.host) : 0;
            a.dlen[i] = pkts[i] ? len[i] : 0;
        }
    }
    for (uint32_t i = 0; i < n; i++) {
        a.ptrs[i] = pkts[i];
        a.lens[i] = len[i];
    }
    a.n = n;
    a.compute = compute;
    a.flags = flags;
    a.status = out8;
    a.csums = csums;
    // The kernel never writes the frames: a fill returns the checks in the
    // records and gcs_wait writes them into the frames from the host; a
    // verify's tcp_in.c:1237 side effect is applied there too.  For frames in
    // a registered region that saves the kernel's writes over PCIe and the
    // release + ack round trip an in-place completion waits for (64 x 1500 B,
    // tools/tx_async_probe.py: send_pkts blocked 9.2 us in place vs ~6 us with
    // host-side checks).
    uint32_t got = 0;
    int rc = ctx->server->post(frames_d, bytes, a.off.data(), a.dlen.data(), n, compute,
                               compute ? (uint32_t)GCS_CF_NO_INPLACE : 0u, a.st.data(),
                               compute ? a.cs.data() : nullptr, /*in_place=*/false,
                               a.staged ? (a.stage_dev ? gcs::kModeDevFrames : 0u)
                                        : (reg.uncached ? gcs::kModeUncachedFrames : 0u),
                               &got);
    if (rc) return rc;
    a.q = got;
    a.pending = true;
    *ticket = got;
    return GCS_OK;
}

}  // namespace

int gcs_compute_ptrs_async(gcs_ctx* ctx, uint8_t* const* pkts, const uint16_t* len, uint32_t n,
                           uint8_t* status, uint32_t* csums, uint64_t* ticket)
try {
    if (!ctx || !ticket || (n && (!pkts || !len)))
        return GCS_EINVAL;
    *ticket = 0;
    if (n == 0)
        return GCS_OK;
    if (ctx->faults && fault("compute_async"))   // test-only (plugin async-post failure)
        return hip_fail(hipErrorLaunchFailure, "injected (compute_async)");
    return post_async(ctx, pkts, len, n, true, 0u, status, csums, ticket);
} GCS_CATCH

int gcs_verify_ptrs_async(gcs_ctx* ctx, uint8_t* const* pkts, const uint16_t* len, uint32_t n,
                          uint8_t* verdict, uint32_t flags, uint64_t* ticket)
try {
    if (!ctx || !ticket || (n && (!pkts || !len || !verdict)))
        return GCS_EINVAL;
    *ticket = 0;
    if (n == 0)
        return GCS_OK;
    if (ctx->faults && (fault("verify_async") || fault("verify_ptrs")))   // test-only
        return hip_fail(hipErrorLaunchFailure, "injected (verify_async)");
    return post_async(ctx, pkts, len, n, false, flags, verdict, nullptr, ticket);
} GCS_CATCH

int gcs_wait(gcs_ctx* ctx, uint64_t ticket)
try {
    if (!ctx)
        return GCS_EINVAL;
    if (ticket == 0)
        return GCS_OK;
    return async_wait(ctx, (uint32_t)ticket);
} GCS_CATCH

int gcs_verify_ptrs(gcs_ctx* ctx, uint8_t* const* pkts, const uint16_t* len, uint32_t n,
                    uint8_t* verdict, uint32_t flags)
try {
    if (ctx && ctx->faults && n && fault("verify_ptrs"))   // test-only (plugin RX failure)
        return hip_fail(hipErrorLaunchFailure, "injected (verify_ptrs)");
    return run_host_batch(ctx, nullptr, nullptr, pkts, len, n, verdict, nullptr, flags, false);
} GCS_CATCH

int gcs_compute_ptrs(gcs_ctx* ctx, uint8_t* const* pkts, const uint16_t* len, uint32_t n,
                     uint8_t* status, uint32_t* csums)
try {
    if (ctx && ctx->faults && n && fault("compute_ptrs"))  // test-only (plugin TX failure)
        return hip_fail(hipErrorLaunchFailure, "injected (compute_ptrs)");
    return run_host_batch(ctx, nullptr, nullptr, pkts, len, n, status, csums, 0u, true);
} GCS_CATCH

}  // extern "C"
