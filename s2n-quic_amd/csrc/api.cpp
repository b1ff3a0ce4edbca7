// api.cpp — host runtime behind include/qpp.h: contexts (one per GPU), the device key table, per-packet
// trait mirrors (a batch of one on the GPU), the batch entry points and the host-memory pipeline.  No CPU
// fallback exists: every byte of payload is sealed/opened by the HIP kernels; without a gfx950 device the
// calls fail with QPP_DEVICE_ERROR.
//
// Asynchrony rules (DESIGN.md §2 "Key lifetime"):
//   * every stream a batch is enqueued on gets a StreamState: its own plan scratch (two streams of one context never
//     share counts/perm/work) and an event recorded after its latest batch;
//   * key records reach HBM on the context's key stream (one install launch per flush, over a slot list, never a range
//     that could rewrite a live neighbour) and a `keys_ready` event; a batch on any stream first waits (device side)
//     for the latest install it has not yet waited for.  The host never blocks on data batches to install a key;
//   * a freed key's slot is retired in stream order on the retire stream: freed slots collect in a pending list that
//     is flushed before the next batch, key install or synchronisation (or once it holds kRetireFlush slots): the
//     retire stream waits for every StreamState's last event, one memset per run of consecutive slots zeroes their
//     device records, and one
//     "retired" event marks them; the slots are reused only once that completed.  (A rotation of 4096 keys used to
//     cost 4096 memset launches.)
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <deque>
#include <map>
#include <mutex>
#include <unordered_map>
#include <string>
#include <vector>

#include "qpp_internal.h"

using namespace qpp;

namespace {

struct StreamState {
    hipStream_t stream = nullptr;
    PlanBuffers plan{};
    uint32_t plan_n_cap = 0, plan_key_cap = 0;
    hipEvent_t last = nullptr;  // after this stream's latest batch
    bool used = false;          // `last` has been recorded at least once
    uint64_t key_gen = 0;       // the latest key install this stream has waited for
    // FIPS-mode nonce-order gate scratch (fips.hip): sort keys, scans, the gated descriptor copy, rocPRIM temp
    void *fips_buf = nullptr;
    size_t fips_bytes = 0;
    uint32_t fips_n_cap = 0;
    uint32_t *fips_refused = nullptr;  // device word: packets the gate refused (txq flushes report it)
    uint32_t *rx_scratch = nullptr;    // fused receive kernel (quad.hip): barrier, per-key counts / cursors, work items
    uint32_t rx_scratch_keys = 0;      // the key_cap it is sized for
    // a mixed-suite batch's ChaCha20 kernel runs on this side stream beside the AES kernel (fork after the plan, join
    // before the batch's last event): its workgroups fill the CUs the AES kernel's last workgroups leave
    hipStream_t side = nullptr;
    hipEvent_t fork_ev = nullptr, join_ev = nullptr;
};

struct KStage {
    uint8_t *h = nullptr, *d = nullptr;
    size_t cap = 0;
    size_t pending = 0;          // bytes of key records / secrets in h, zeroized once the job's copy is done
    hipEvent_t free_ev = nullptr;  // recorded on the key stream after the last job that reads this stage
    bool used = false;
};

struct Retired {
    std::vector<uint32_t> slots;
    hipEvent_t done;  // the zeroing of these device records (retire stream) has completed
};
constexpr size_t kRetireFlush = 4096;  // pending retirements that force a flush from qpp_key_free itself

// One slot of the host pipeline: device buffers for one chunk in flight, and the events that order its reuse.
struct PipeSlot {
    uint8_t *arena = nullptr;  // chunk span of the arena
    qpp_pkt *descs = nullptr;
    uint8_t *masks = nullptr;
    int8_t *status = nullptr;
    hipEvent_t h2d = nullptr, comp = nullptr, d2h = nullptr;
    bool busy = false;  // d2h has been recorded (the next user waits for it)
};

struct HostPipe {
    // Buffers for chunks of up to 256 Ki packets.  Unless the geometry is set (qpp_ctx_set_host_pipe), a batch is cut
    // into ~16 chunks of 64-256 Ki packets, and at least 64 packets per live AES key (one full wave-item each): with
    // 4096 keys, 64 Ki-packet chunks ran the C5 pipeline at 76 ms/step instead of 62; with one key, 256 Ki-packet
    // chunks made a 1 Mi-packet batch 33 ms instead of 29 (pipeline fill and drain).  profiles/r02_e2e.jsonl
    size_t chunk_packets = 262144, chunk_bytes = 384u << 20, nslots = 4;
    bool auto_chunk = true;
    hipStream_t h2d = nullptr, comp = nullptr, d2h = nullptr;
    std::vector<PipeSlot> slots;
    size_t next = 0;
    uint64_t next_ticket = 1;
    std::map<uint64_t, hipEvent_t> tickets;
};

}  // namespace

struct qpp_ctx {
    int device = 0;
    uint32_t n_cu = 0;  // compute units (AES work-item sizing)
    uint32_t burst_max = kBurstMaxDefault;  // AES batches up to this size take the wave-per-packet kernel
    int aes_kernel = 0;  // QPP_AES_KERNEL_*: 0 = chosen per batch (aes_path)
    hipStream_t stream = nullptr;
    hipStream_t kstream = nullptr;  // key installs / derivations
    hipStream_t rstream = nullptr;  // key retirements (zeroization behind in-flight batches)
    hipEvent_t keys_ready = nullptr;
    uint64_t key_gen = 0;           // installs so far (keys_ready marks the latest)
    // device key table + host mirror
    DevKey *d_keys = nullptr;
    uint32_t key_cap = 0;
    PowTables pow{nullptr, 0};  // burst power tables of slots < pow.cap (grown with the key table, <= kPowSlots)
    std::vector<DevKey> h_keys;
    std::vector<uint8_t> dirty_flag;
    std::vector<uint32_t> dirty;          // slots whose host record must be installed before the next launch
    std::vector<uint32_t> free_slots;     // reusable now
    std::deque<Retired> retired;          // reusable once `done` has completed
    std::vector<uint32_t> retire_pending; // freed, host copy zeroized, device zeroing not yet enqueued
    uint32_t retired_slots = 0;           // slots in `retired`
    uint32_t live_by_suite[4] = {0, 0, 0, 0};  // live packet keys per suite: which kernels a batch can need
    uint32_t hdr_live_by_suite[4] = {0, 0, 0, 0};  // live header-key-only records per suite (the fused ChaCha receive)
    uint32_t live_slot_xor = 0;                  // XOR of the live packet keys' slots: THE slot when only one is live
    bool fips = false;                           // qpp_ctx_set_fips: AES packet keys created now seal in FIPS mode
    uint32_t fips_live = 0;                      // live FIPS keys: seal batches run the nonce-order gate
    // The nonce-order state lives in the device key records and the gate reads and advances it without atomics, so
    // the gates of all streams run one after another in submission order: each gate's stream waits for this event
    // (recorded behind the previous gate, on whatever stream that ran) -- two txq flushes in flight on different
    // streams could otherwise both pass a repeated packet number, or a later flush refuse an earlier one's packets.
    hipEvent_t fips_order = nullptr;
    bool fips_order_used = false;
    uint32_t next_slot = 0;
    // per-stream state (plan scratch, last-batch event); [0] is the context stream
    std::vector<StreamState *> streams;
    // every other stream the caller handed this context or got from it (qpp_stream_create; a non-null stream of
    // qpp_memcpy_*, qpp_memset_d, qpp_event_record, qpp_stream_wait_event) until qpp_stream_destroy: qpp_ctx_synchronize
    // waits for these too (a copy-only stream has no StreamState)
    std::vector<hipStream_t> user_streams;
    std::vector<hipEvent_t> event_pool;
    // per-packet staging (pinned, zero-copy) and key staging (pinned + device)
    uint8_t *d_stage = nullptr, *h_stage = nullptr;
    uint8_t *v_stage = nullptr;  // device view of the pinned h_stage (zero-copy per-packet calls)
    size_t stage_cap = 0;
    // two pinned key stages (+ device twins), used alternately by the key-stream jobs (installs, derivations): a
    // job waits only for the previous job of ITS stage (an event), never for the key stream as a whole
    KStage kstage[2];
    int kstage_next = 0;
    HostPipe *pipe = nullptr;
    std::vector<qpp_txq *> servers;  // transmit queues with a persistent server kernel (qpp_txq_create_persistent)
    std::vector<qpp_txq *> txqs;     // every transmit queue of the context (their flush streams: ctx_streams)
    // The packet server: a persistent queue of the context's own (kPktWgs workgroups, created on the first per-packet
    // call) through which qpp_seal / qpp_open run without a kernel launch; qpp_ctx_set_packet_server, QPP_PACKET_SERVER
    qpp_txq *pkt_q = nullptr;
    bool pkt_server = true;
    uint64_t pkt_calls = 0, pkt_starts = 0;  // qpp_ctx_packet_server_info (starts of freed servers in pkt_starts)
    uint32_t *d_connmap = nullptr;    // qpp_ctx_set_conn_keys: connection -> key slot (device)
    size_t connmap_cap = 0, connmap_n = 0;
    // its pinned staging copy (the caller's array is pageable: HIP does not promise an async copy from it has read it
    // when the call returns), reused once connstage_ev shows the previous copy done
    uint32_t *h_connstage = nullptr;
    size_t connstage_cap = 0;
    hipEvent_t connstage_ev = nullptr;
    bool connstage_used = false;
    uint32_t *d_diag = nullptr;  // device counters: [0] fused-receive workgroups that left on a barrier timeout
    std::string last_error;
};

struct qpp_key {
    qpp_ctx *ctx = nullptr;
    int suite = 0;
    uint32_t slot = 0;
    bool has_secret = false;
    uint8_t secret[48] = {0};
    uint8_t key[32] = {0};
    uint8_t iv[12] = {0};
    uint8_t hp[32] = {0};
};

// HeaderKey (header_key.rs:7-63): owned independently of any packet key; its own device slot (live = 2) holds only
// the header-protection key schedule.
struct qpp_header_key {
    qpp_ctx *ctx = nullptr;
    int suite = 0;
    uint32_t slot = 0;
    uint8_t hp[32] = {0};
};

namespace {

bool fail(qpp_ctx *ctx, hipError_t e, const char *what) {
    if (e == hipSuccess) return false;
    if (ctx) ctx->last_error = std::string(what) + ": " + hipGetErrorString(e);
    return true;
}
#define HIP_TRY(ctx, expr)                                      \
    do {                                                        \
        if (fail((ctx), (expr), #expr)) return QPP_DEVICE_ERROR; \
    } while (0)
#define RC_TRY(expr)          \
    do {                      \
        int rc_ = (expr);     \
        if (rc_) return rc_;  \
    } while (0)

// Persistent transmit-queue servers (defined with qpp_txq below).  A server kernel never ends on its own while
// flushes keep coming, so every device-wide wait first stops them (servers_stop), and key retirement first waits
// for their flushes in flight (servers_quiesce).
int servers_stop(qpp_ctx *ctx);
int servers_quiesce(qpp_ctx *ctx);
uint32_t servers_cu(const qpp_ctx *ctx);
// ---------------------------------------------------------------- resident servers of a device (process-wide)
// Persistent server kernels -- transmit-queue servers and the contexts' packet servers -- hold whole CUs while they run,
// and their streams share the device's greatest-priority hardware queues.  One registry per device, over every context
// of the process:
//   * cu_avail counts the workgroups of EVERY resident server of the device, so a full-chip grid -- above all the fused
//     receive's, whose grid barriers need every workgroup resident at once -- is sized for the CUs really left;
//   * fused receives of the device run one after another (each waits, device side, for the previous one: two on two
//     streams would split the CUs and both time out), and a server launch waits for the latest fused receive (a server
//     starting while a receive's workgroups are being dispatched would take CUs the receive's grid counted on);
//   * at most GPU_MAX_HW_QUEUES (default 4) servers are resident per device: the runtime maps the streams of one
//     priority level onto that many hardware queues, and a server launched onto a hardware queue a resident server
//     holds would wait for that server's idle exit.  A queue finding no free server slot takes the launched path (a
//     transmit-queue flush) or launches the per-packet kernel (the packet server's callers).
struct DevServers {
    std::mutex mu;
    std::vector<qpp_txq *> queues;  // the persistent queues of every context on the device
    hipEvent_t rx_tail = nullptr;   // recorded behind the device's latest fused receive
    std::vector<std::pair<void *, bool>> parked;  // buffers (pinned: true) freed once no server is resident (release)
    size_t parked_bytes = 0;
    // the device's eviction word (16 B, coherent pinned memory; host view / device view): non-zero makes every resident
    // server of the device leave at its next poll without a complete flush (release past the parked bound)
    uint32_t *h_evict = nullptr, *v_evict = nullptr;
    uint64_t evictions = 0, oneshots = 0;  // qpp_dev_server_evictions
};
// past this many parked bytes per device, release evicts the device's resident servers and frees; env QPP_PARKED_MAX_MB
size_t parked_max() {
    static const size_t v = [] {
        const char *e = getenv("QPP_PARKED_MAX_MB");
        return e ? (size_t)strtoull(e, nullptr, 10) << 20 : size_t(2) << 30;
    }();
    return v;
}
DevServers &dev_servers(int device) {
    static DevServers regs[64];
    return regs[(unsigned)device & 63u];
}
uint32_t server_slots() {
    static const uint32_t n = [] {
        const char *e = getenv("GPU_MAX_HW_QUEUES");
        const unsigned long v = e ? strtoul(e, nullptr, 10) : 4ul;
        return (uint32_t)(v ? std::min(v, 32ul) : 4ul);
    }();
    return n;
}
uint32_t resident_wgs_locked(const DevServers &r);  // (with qpp_txq below)
// Key::encrypt / Key::decrypt of one packet through the context's packet server (defined with qpp_txq below);
// *handled = false: the call is not one the server takes (FIPS seal, packet over kPktRing, server off) -- launch it
int packet_server_run(const qpp_key *k, bool seal, uint64_t pn, const uint8_t *header, size_t header_len,
                      const uint8_t *payload, size_t payload_len, uint8_t *out, uint8_t *tag_out, int8_t *status_out,
                      bool *handled);
// HeaderKey::*_header_protection_mask of one sample through the packet server (*handled = false: server off)
int packet_server_mask(qpp_ctx *ctx, uint32_t slot, const uint8_t *sample, uint8_t mask[5], bool *handled);
// CUs a full-chip kernel (one workgroup per CU) should size its grid for: those of the device's resident servers --
// every context's (servers_cu) -- are taken
uint32_t cu_avail(const qpp_ctx *ctx) {
    const uint32_t r = servers_cu(ctx);
    return ctx->n_cu > r ? ctx->n_cu - r : 1u;
}
// Memory without device-wide waits.  hipFree, hipHostFree, hipHostUnregister and hipDeviceSynchronize wait for EVERY
// stream of the device -- a resident server's too, and a server leaves only on its idle timeout (200 ms by default),
// or never while its flushes keep coming.  Measured beside a resident kernel (tools/diag/free_sync.hip,
// profiles/r05/r05v): each of those calls took 1950 ms next to a 2-s kernel; hipMalloc, hipHostMalloc, hipMallocAsync,
// hipFreeAsync, hipStreamDestroy and hipEventDestroy did not wait.  (The stream-ordered allocator was tried for device
// memory and corrupted batch buffers in the fuzz test -- 6-8 of 44 seeds, with or without device-wide synchronizes,
// 0 of 44 with hipMalloc / hipFree: profiles/r05/r05v/fuzzab.txt -- so it is not used.)  Hence:
//   * device and pinned buffers are freed at once only while no server of the device is resident (any context's,
//     this one's included), else parked in the device registry and freed by the next free, synchronize or destroy of
//     any context that finds none resident (release); parked memory is never reused before that hipFree, so work
//     still reading it is unaffected, and no server is stopped to free memory it does not read;
//   * a context's synchronize waits for every stream of the context (ctx_sync), never the device.
int quiet_for_free(qpp_ctx *ctx) { return servers_stop(ctx); }
void release(qpp_ctx *ctx, void *p, bool pinned);  // (with the registry's users below)
void hfree(qpp_ctx *ctx, void *p) { release(ctx, p, true); }
void dfree(qpp_ctx *ctx, void *p) {
    if (p) release(ctx, p, false);
}
// Sizes of the library's device and pinned allocations, so that release() counts parked bytes exactly (hipMemPtrGetInfo
// does not size every pinned buffer: ADVICE r5).  Process-wide: a buffer may be released by another context's call.
std::mutex g_size_mu;
std::unordered_map<void *, size_t> g_sizes;
void note_size(void *p, size_t bytes) {
    std::lock_guard<std::mutex> lk(g_size_mu);
    g_sizes[p] = bytes;
}
size_t take_size(void *p) {
    std::lock_guard<std::mutex> lk(g_size_mu);
    auto it = g_sizes.find(p);
    if (it == g_sizes.end()) return 0;
    const size_t b = it->second;
    g_sizes.erase(it);
    return b;
}
template <class T>
hipError_t dmalloc(qpp_ctx *, T **p, size_t bytes) {
    const hipError_t e = hipMalloc((void **)p, bytes ? bytes : 1);
    if (e == hipSuccess) note_size((void *)*p, bytes ? bytes : 1);
    return e;
}
template <class T>
hipError_t hmalloc(T **p, size_t bytes, unsigned flags) {
    const hipError_t e = hipHostMalloc((void **)p, bytes ? bytes : 1, flags);
    if (e == hipSuccess) note_size((void *)*p, bytes ? bytes : 1);
    return e;
}

bool valid_suite(int s) {
    return s == QPP_SUITE_TLS_AES_128_GCM_SHA256 || s == QPP_SUITE_TLS_AES_256_GCM_SHA384 ||
           s == QPP_SUITE_TLS_CHACHA20_POLY1305_SHA256;
}
bool is_aes(int suite) { return suite != QPP_SUITE_TLS_CHACHA20_POLY1305_SHA256; }
constexpr uint32_t kAesSuites = (1u << QPP_SUITE_TLS_AES_128_GCM_SHA256) | (1u << QPP_SUITE_TLS_AES_256_GCM_SHA384);

hipEvent_t get_event(qpp_ctx *ctx) {
    if (!ctx->event_pool.empty()) {
        hipEvent_t e = ctx->event_pool.back();
        ctx->event_pool.pop_back();
        return e;
    }
    hipEvent_t e = nullptr;
    if (hipEventCreateWithFlags(&e, hipEventDisableTiming) != hipSuccess) return nullptr;
    return e;
}
void put_event(qpp_ctx *ctx, hipEvent_t e) {
    if (e) ctx->event_pool.push_back(e);
}

const std::vector<hipStream_t> &txq_streams(const qpp_txq *q);  // (with qpp_txq below)
// every stream the context's work runs on (the resident servers' excepted): its own, each batch stream's (with its
// ChaCha side stream, and the transmit queues' flush streams, which are batch streams), the host pipeline's
std::vector<hipStream_t> ctx_streams(const qpp_ctx *ctx) {
    std::vector<hipStream_t> v;
    for (hipStream_t s : {ctx->stream, ctx->kstream, ctx->rstream})
        if (s) v.push_back(s);
    for (const StreamState *st : ctx->streams) {
        if (st->stream != ctx->stream) v.push_back(st->stream);
        if (st->side) v.push_back(st->side);
    }
    if (ctx->pipe)
        for (hipStream_t s : {ctx->pipe->h2d, ctx->pipe->comp, ctx->pipe->d2h})
            if (s) v.push_back(s);
    for (const qpp_txq *q : ctx->txqs)  // (zero-copy flushes run on them without a stream state; read the key table)
        for (hipStream_t s : txq_streams(q)) v.push_back(s);
    for (hipStream_t s : ctx->user_streams) v.push_back(s);
    return v;
}
// remember a caller's stream (see qpp_ctx::user_streams); returns it (NULL: the context stream)
hipStream_t user_stream(qpp_ctx *ctx, void *stream) {
    hipStream_t s = (hipStream_t)stream;
    if (!s || s == ctx->stream) return ctx->stream;
    if (std::find(ctx->user_streams.begin(), ctx->user_streams.end(), s) == ctx->user_streams.end())
        ctx->user_streams.push_back(s);
    return s;
}
int ctx_sync(qpp_ctx *ctx) {
    for (hipStream_t s : ctx_streams(ctx)) HIP_TRY(ctx, hipStreamSynchronize(s));
    return QPP_OK;
}

// (the plan's stream has been synchronized)
void free_plan(qpp_ctx *ctx, PlanBuffers &p) {
    for (void *b : {(void *)p.counts, (void *)p.cursor, (void *)p.istart, (void *)p.perm, (void *)p.kq,
                    (void *)p.work, (void *)p.n_work})
        dfree(ctx, b);
    p = PlanBuffers{};
}
void free_stream_state(qpp_ctx *ctx, StreamState *st) {
    hipStreamSynchronize(st->stream);
    if (st->side) hipStreamSynchronize(st->side);
    free_plan(ctx, st->plan);
    dfree(ctx, st->fips_buf);
    dfree(ctx, st->fips_refused);
    dfree(ctx, st->rx_scratch);
    if (st->side) hipStreamDestroy(st->side);
    if (st->fork_ev) hipEventDestroy(st->fork_ev);
    if (st->join_ev) hipEventDestroy(st->join_ev);
    if (st->last) hipEventDestroy(st->last);
    delete st;
}

StreamState *stream_state(qpp_ctx *ctx, hipStream_t s) {
    for (StreamState *st : ctx->streams)
        if (st->stream == s) return st;
    StreamState *st = new StreamState();
    st->stream = s;
    if (hipEventCreateWithFlags(&st->last, hipEventDisableTiming) != hipSuccess) {
        delete st;
        return nullptr;
    }
    ctx->streams.push_back(st);
    return st;
}

// Before enqueueing a batch on st: its launches must see every key installed so far (device-side wait).
int see_keys(qpp_ctx *ctx, StreamState *st) {
    if (st->key_gen == ctx->key_gen) return QPP_OK;
    HIP_TRY(ctx, hipStreamWaitEvent(st->stream, ctx->keys_ready, 0));
    st->key_gen = ctx->key_gen;
    return QPP_OK;
}

// After enqueueing a batch on st: remember where it ends (key retirement orders behind it).
int note_work(qpp_ctx *ctx, StreamState *st) {
    HIP_TRY(ctx, hipEventRecord(st->last, st->stream));
    st->used = true;
    return QPP_OK;
}

// The stream state of a batch call on `stream` (NULL: the context stream), ready for launches.
int batch_stream(qpp_ctx *ctx, void *stream, StreamState **out) {
    StreamState *st = stream_state(ctx, stream ? (hipStream_t)stream : ctx->stream);
    if (!st) return QPP_DEVICE_ERROR;
    RC_TRY(see_keys(ctx, st));
    *out = st;
    return QPP_OK;
}

int grow_keys(qpp_ctx *ctx, uint32_t need) {
    if (need <= ctx->key_cap) return QPP_OK;
    uint32_t cap = std::max<uint32_t>(64, ctx->key_cap);
    while (cap < need) cap *= 2;
    DevKey *nk = nullptr;
    RC_TRY(servers_stop(ctx));  // they hold the old table's address
    RC_TRY(ctx_sync(ctx));      // no batch may still read the old table
    HIP_TRY(ctx, dmalloc(ctx, &nk, sizeof(DevKey) * cap));
    // Stream-ordered and waited for: a plain hipMemset runs on the null stream, which does not order against the
    // context's non-blocking streams (a batch could read the table before it is zeroed).
    HIP_TRY(ctx, hipMemsetAsync(nk, 0, sizeof(DevKey) * cap, ctx->kstream));
    if (ctx->d_keys) {
        HIP_TRY(ctx, hipMemcpyAsync(nk, ctx->d_keys, sizeof(DevKey) * ctx->key_cap, hipMemcpyDeviceToDevice,
                                    ctx->kstream));
        HIP_TRY(ctx, hipMemsetAsync(ctx->d_keys, 0, sizeof(DevKey) * ctx->key_cap, ctx->kstream));
    }
    const uint32_t pcap = std::min<uint32_t>(cap, kPowSlots);
    uint8_t *np = ctx->pow.base;
    if (pcap > ctx->pow.cap) {  // the precomputed tables of the slots so far move along
        HIP_TRY(ctx, dmalloc(ctx, &np, (size_t)pcap * kPowBytes));
        if (ctx->pow.cap) {
            HIP_TRY(ctx, hipMemcpyAsync(np, ctx->pow.base, (size_t)ctx->pow.cap * kPowBytes, hipMemcpyDeviceToDevice,
                                        ctx->kstream));
            // powers of each key's H: zeroized before the old buffer goes back to the allocator, like the records
            HIP_TRY(ctx, hipMemsetAsync(ctx->pow.base, 0, (size_t)ctx->pow.cap * kPowBytes, ctx->kstream));
        }
    }
    HIP_TRY(ctx, hipStreamSynchronize(ctx->kstream));
    dfree(ctx, ctx->d_keys);
    if (np != ctx->pow.base) {
        dfree(ctx, ctx->pow.base);
        ctx->pow = PowTables{np, pcap};
    }
    ctx->d_keys = nk;
    ctx->h_keys.resize(cap);
    ctx->dirty_flag.resize(cap, 0);
    ctx->key_cap = cap;
    return QPP_OK;
}

// The key stage for the next key-stream job, with room for `bytes`: the stage the previous job did not use, once
// ITS previous job has read it (host wait on that job's event only -- the other stage's job, e.g. the install that
// flush_keys just queued, keeps running).  The caller records release_kstage after enqueueing its copies.
int take_kstage(qpp_ctx *ctx, size_t bytes, KStage **out) {
    KStage &k = ctx->kstage[ctx->kstage_next];
    ctx->kstage_next ^= 1;
    if (k.used) HIP_TRY(ctx, hipEventSynchronize(k.free_ev));
    k.used = false;
    if (k.pending) secure_zero(k.h, k.pending);
    k.pending = 0;
    if (!k.free_ev) HIP_TRY(ctx, hipEventCreateWithFlags(&k.free_ev, hipEventDisableTiming));
    if (bytes > k.cap) {
        size_t cap = std::max<size_t>(1 << 16, k.cap);
        while (cap < bytes) cap *= 2;
        dfree(ctx, k.d);  // (its last job, the previous user of this stage, is done)
        if (k.h) { secure_zero(k.h, k.cap); hfree(ctx, k.h); }
        k.d = nullptr;
        k.h = nullptr;
        k.cap = 0;
        HIP_TRY(ctx, dmalloc(ctx, &k.d, cap));
        HIP_TRY(ctx, hmalloc(&k.h, cap, hipHostMallocDefault));
        k.cap = cap;
    }
    *out = &k;
    return QPP_OK;
}
// after the job's last read of the stage was enqueued on the key stream; `pending` bytes of h are zeroized later
int release_kstage(qpp_ctx *ctx, KStage *k, size_t pending) {
    HIP_TRY(ctx, hipEventRecord(k->free_ev, ctx->kstream));
    k->used = true;
    k->pending = pending;
    return QPP_OK;
}

int flush_retire(qpp_ctx *ctx);

// Installs every pending host record on the device: one copy + one install launch on the key stream, then the
// keys_ready event that the next batch on every stream waits for (device side; H and V[m] included).
int flush_keys(qpp_ctx *ctx) {
    RC_TRY(flush_retire(ctx));
    if (ctx->dirty.empty()) return QPP_OK;
    const uint32_t n = (uint32_t)ctx->dirty.size();
    const size_t rec = sizeof(DevKey) * n, slots = 4 * (size_t)n;
    KStage *k = nullptr;
    RC_TRY(take_kstage(ctx, rec + slots, &k));
    for (uint32_t i = 0; i < n; i++) {
        memcpy(k->h + sizeof(DevKey) * i, &ctx->h_keys[ctx->dirty[i]], sizeof(DevKey));
        ctx->dirty_flag[ctx->dirty[i]] = 0;
    }
    memcpy(k->h + rec, ctx->dirty.data(), slots);
    hipStream_t s = ctx->kstream;
    HIP_TRY(ctx, hipMemcpyAsync(k->d, k->h, rec + slots, hipMemcpyHostToDevice, s));
    HIP_TRY(ctx, launch_key_install(ctx->d_keys, (const uint32_t *)(k->d + rec), (const DevKey *)k->d, n, ctx->pow, s));
    HIP_TRY(ctx, hipMemsetAsync(k->d, 0, rec, s));
    HIP_TRY(ctx, hipEventRecord(ctx->keys_ready, s));
    ctx->key_gen++;
    ctx->dirty.clear();
    // the pinned copy of the records is zeroized when the stage is next taken (its copy is done by then)
    return release_kstage(ctx, k, rec);
}

void mark_dirty(qpp_ctx *ctx, uint32_t slot) {
    if (!ctx->dirty_flag[slot]) {
        ctx->dirty_flag[slot] = 1;
        ctx->dirty.push_back(slot);
    }
}

int ensure_plan(qpp_ctx *ctx, StreamState *st, uint32_t n) {
    if (n <= st->plan_n_cap && ctx->key_cap <= st->plan_key_cap) return QPP_OK;
    HIP_TRY(ctx, hipStreamSynchronize(st->stream));  // the old scratch is no longer read
    PlanBuffers &p = st->plan;
    free_plan(ctx, p);
    st->plan_n_cap = st->plan_key_cap = 0;
    const uint32_t ncap = std::max(n, st->plan_n_cap), kcap = ctx->key_cap;
    HIP_TRY(ctx, dmalloc(ctx, &p.counts, sizeof(uint32_t) * kcap));
    // zeroed on the batch's own stream: plan_hist on this stream follows it.  (A plain hipMemset goes to the null
    // stream, which does not order against non-blocking streams: with recycled device memory plan_hist then counted
    // on top of stale words and the scatter wrote past perm[] -- an illegal address under two concurrent streams.)
    HIP_TRY(ctx, hipMemsetAsync(p.counts, 0, sizeof(uint32_t) * kcap, st->stream));  // plan_scan re-zeroes it after each plan
    HIP_TRY(ctx, dmalloc(ctx, &p.cursor, sizeof(uint32_t) * kcap));
    HIP_TRY(ctx, dmalloc(ctx, &p.istart, sizeof(uint32_t) * 2 * (kcap + 1)));
    HIP_TRY(ctx, dmalloc(ctx, &p.perm, sizeof(uint32_t) * std::max<uint32_t>(ncap, 1)));
    HIP_TRY(ctx, dmalloc(ctx, &p.kq, sizeof(uint32_t) * std::max<uint32_t>(ncap, 1)));
    HIP_TRY(ctx, dmalloc(ctx, &p.work, sizeof(WorkItem) * (plan_max_work(ncap, kcap, kMinPacketsPerItem) + 1)));
    HIP_TRY(ctx, dmalloc(ctx, &p.n_work, 8 * sizeof(uint32_t)));
    HIP_TRY(ctx, hipMemsetAsync(p.n_work, 0, 8 * sizeof(uint32_t), st->stream));  // (meta[6] is a running count)
    st->plan_n_cap = ncap;
    st->plan_key_cap = kcap;
    return QPP_OK;
}

// FIPS gate scratch for batches of up to n packets on st (plus its refused-packet counter)
int ensure_fips(qpp_ctx *ctx, StreamState *st, uint32_t n) {
    if (!st->fips_refused) {
        HIP_TRY(ctx, dmalloc(ctx, &st->fips_refused, 256));
        HIP_TRY(ctx, hipMemsetAsync(st->fips_refused, 0, 4, st->stream));
    }
    if (n <= st->fips_n_cap) return QPP_OK;
    HIP_TRY(ctx, hipStreamSynchronize(st->stream));  // the old scratch is no longer read
    dfree(ctx, st->fips_buf);
    st->fips_buf = nullptr;
    st->fips_n_cap = 0;
    const uint32_t cap = std::max<uint32_t>(n, 1024);
    st->fips_bytes = fips_scratch_bytes(cap);
    HIP_TRY(ctx, dmalloc(ctx, &st->fips_buf, st->fips_bytes));
    st->fips_n_cap = cap;
    return QPP_OK;
}

// FIPS mode: the descriptors the seal kernels read instead of descs (refused packets skipped; status / refused count
// written).  Unchanged when no FIPS key is live.
int fips_gate(qpp_ctx *ctx, StreamState *st, const qpp_pkt *&descs, uint32_t n, int8_t *status, uint32_t *refused) {
    if (!ctx->fips_live || !n) return QPP_OK;
    RC_TRY(ensure_fips(ctx, st, n));
    if (!ctx->fips_order) HIP_TRY(ctx, hipEventCreateWithFlags(&ctx->fips_order, hipEventDisableTiming));
    if (ctx->fips_order_used) HIP_TRY(ctx, hipStreamWaitEvent(st->stream, ctx->fips_order, 0));
    qpp_pkt *gated = nullptr;
    HIP_TRY(ctx, launch_fips_gate(ctx->d_keys, ctx->key_cap, descs, n, st->fips_buf, st->fips_bytes, &gated, status,
                                  refused, st->stream));
    HIP_TRY(ctx, hipEventRecord(ctx->fips_order, st->stream));
    ctx->fips_order_used = true;
    descs = gated;
    return QPP_OK;
}

int ensure_stage(qpp_ctx *ctx, size_t bytes) {
    if (bytes <= ctx->stage_cap) return QPP_OK;
    size_t cap = std::max<size_t>(4096, ctx->stage_cap);
    while (cap < bytes) cap *= 2;
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    dfree(ctx, ctx->d_stage);
    hfree(ctx, ctx->h_stage);
    ctx->d_stage = ctx->h_stage = ctx->v_stage = nullptr;
    ctx->stage_cap = 0;
    HIP_TRY(ctx, dmalloc(ctx, &ctx->d_stage, cap));
    HIP_TRY(ctx, hmalloc(&ctx->h_stage, cap, hipHostMallocDefault));
    void *v = nullptr;
    HIP_TRY(ctx, hipHostGetDevicePointer(&v, ctx->h_stage, 0));
    ctx->v_stage = (uint8_t *)v;
    ctx->stage_cap = cap;
    return QPP_OK;
}

// A slot for a new key: a retired slot whose zeroing has completed, else a fresh one.
int alloc_slot(qpp_ctx *ctx, uint32_t *out) {
    RC_TRY(flush_retire(ctx));
    while (!ctx->retired.empty()) {
        const hipError_t q = hipEventQuery(ctx->retired.front().done);
        if (q == hipErrorNotReady) break;
        if (fail(ctx, q, "retired slot event")) return QPP_DEVICE_ERROR;
        Retired &r = ctx->retired.front();
        ctx->free_slots.insert(ctx->free_slots.end(), r.slots.rbegin(), r.slots.rend());
        ctx->retired_slots -= (uint32_t)r.slots.size();
        put_event(ctx, r.done);
        ctx->retired.pop_front();
    }
    if (!ctx->free_slots.empty()) {
        *out = ctx->free_slots.back();
        ctx->free_slots.pop_back();
        return QPP_OK;
    }
    RC_TRY(grow_keys(ctx, ctx->next_slot + 1));
    *out = ctx->next_slot++;
    return QPP_OK;
}

// Zeroizes the slots' device records behind every batch already enqueued on any stream of this context (one launch
// for all pending slots), then queues the slots for reuse (cipher_suite.rs:106-114,189-193 zeroize on drop; here
// "drop" is stream-ordered).  Called before anything new is enqueued, so the retire stream waits only for batches
// enqueued before the keys were freed (and possibly a few after: never too early).
int flush_retire(qpp_ctx *ctx) {
    if (ctx->retire_pending.empty()) return QPP_OK;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    RC_TRY(servers_quiesce(ctx));  // a server flush in flight may still read the freed records
    for (StreamState *st : ctx->streams)
        if (st->used) HIP_TRY(ctx, hipStreamWaitEvent(ctx->rstream, st->last, 0));
    HIP_TRY(ctx, hipStreamWaitEvent(ctx->rstream, ctx->keys_ready, 0));  // behind the slots' own installs
    // one memset per run of consecutive slots (a rotation frees whole batches of keys that were allocated together)
    std::vector<uint32_t> sorted(ctx->retire_pending);
    std::sort(sorted.begin(), sorted.end());
    for (size_t i = 0; i < sorted.size();) {
        size_t j = i + 1;
        while (j < sorted.size() && sorted[j] == sorted[j - 1] + 1) j++;
        HIP_TRY(ctx, hipMemsetAsync(ctx->d_keys + sorted[i], 0, sizeof(DevKey) * (j - i), ctx->rstream));
        if (sorted[i] < ctx->pow.cap) {  // the burst power tables are derived from H: zeroized with the record
            const size_t k = std::min<size_t>(j - i, ctx->pow.cap - sorted[i]);
            HIP_TRY(ctx, hipMemsetAsync(ctx->pow.base + (size_t)sorted[i] * kPowBytes, 0, kPowBytes * k, ctx->rstream));
        }
        i = j;
    }
    hipEvent_t e = get_event(ctx);
    if (!e || hipEventRecord(e, ctx->rstream) != hipSuccess) {
        // no event: wait here instead (a slot must never be reused while a batch may read it)
        put_event(ctx, e);
        HIP_TRY(ctx, hipStreamSynchronize(ctx->rstream));
        ctx->free_slots.insert(ctx->free_slots.end(), ctx->retire_pending.begin(), ctx->retire_pending.end());
        ctx->retire_pending.clear();
        return QPP_OK;
    }
    ctx->retired_slots += (uint32_t)ctx->retire_pending.size();
    ctx->retired.push_back(Retired{std::move(ctx->retire_pending), e});
    ctx->retire_pending.clear();
    return QPP_OK;
}

// Frees a slot: the host copy is zeroized now, the device record behind in-flight work (flush_retire).
void retire_slot(qpp_ctx *ctx, uint32_t slot) {
    secure_zero(&ctx->h_keys[slot], sizeof(DevKey));
    ctx->retire_pending.push_back(slot);
    if (ctx->retire_pending.size() >= kRetireFlush) flush_retire(ctx);
}

// Fills the slot's host record from the key's material and marks it for installation.
int install(qpp_key *k) {
    qpp_ctx *ctx = k->ctx;
    RC_TRY(alloc_slot(ctx, &k->slot));
    DevKey &d = ctx->h_keys[k->slot];
    memset(&d, 0, sizeof d);
    d.suite = (uint32_t)k->suite;
    d.live = 1;
    memcpy(d.iv, k->iv, 12);
    if (k->suite == QPP_SUITE_TLS_CHACHA20_POLY1305_SHA256) {
        memcpy(d.rk, k->key, 32);
        memcpy(d.hp_rk, k->hp, 32);
    } else {
        const size_t kl = suite_key_len(k->suite);
        d.nr = (uint32_t)aes_expand_key(k->key, kl, d.rk);
        d.hp_nr = (uint32_t)aes_expand_key(k->hp, kl, d.hp_rk);
    }
    d.fips = ctx->fips && is_aes(k->suite) ? 1u : 0u;  // no FIPS ChaCha20-Poly1305 (cipher_suite/ring.rs:116-121)
    ctx->fips_live += d.fips;
    mark_dirty(ctx, k->slot);
    ctx->live_by_suite[k->suite]++;
    ctx->live_slot_xor ^= k->slot;
    return QPP_OK;
}

int install_header(qpp_header_key *h) {
    qpp_ctx *ctx = h->ctx;
    RC_TRY(alloc_slot(ctx, &h->slot));
    DevKey &d = ctx->h_keys[h->slot];
    memset(&d, 0, sizeof d);
    d.suite = (uint32_t)h->suite;
    d.live = 2;  // header key only: no packet key, never planned or sealed with
    if (h->suite == QPP_SUITE_TLS_CHACHA20_POLY1305_SHA256) memcpy(d.hp_rk, h->hp, 32);
    else d.hp_nr = (uint32_t)aes_expand_key(h->hp, suite_key_len(h->suite), d.hp_rk);
    ctx->hdr_live_by_suite[h->suite & 3]++;
    mark_dirty(ctx, h->slot);
    return QPP_OK;
}

void derive(qpp_key *k) {
    const size_t hl = suite_hash_len(k->suite), kl = suite_key_len(k->suite);
    hkdf_expand_label(hl, k->secret, "quic key", k->key, kl);
    hkdf_expand_label(hl, k->secret, "quic iv", k->iv, 12);
    hkdf_expand_label(hl, k->secret, "quic hp", k->hp, kl);
}

uint32_t suite_mask(const qpp_ctx *ctx) {
    uint32_t m = 0;
    for (int s = 1; s <= 3; s++)
        if (ctx->live_by_suite[s]) m |= 1u << s;
    return m;
}

// Which AES-GCM kernel serves an n-packet batch: the wave-per-packet burst kernel for small batches; the quad kernel
// (quad.hip: four lanes per packet, one workgroup per CU over a slice of the key-sorted packets, 8-bit GHASH tables
// rebuilt per key segment) when the batch has >= kWaveKernelPacketsPerKey packets per live AES key; else the wave-item
// kernel (aes_gcm.hip: one key per 64-packet wave, 4-bit tables).  QPP_AES_KERNEL=quad|wave forces one of the two
// throughput kernels (A/B).
enum class AesPath { burst, quad, wave };
AesPath aes_path(const qpp_ctx *ctx, uint32_t n) {
    if (n <= ctx->burst_max) return AesPath::burst;
    if (ctx->aes_kernel) return ctx->aes_kernel == QPP_AES_KERNEL_QUAD ? AesPath::quad : AesPath::wave;
    const uint64_t aes_keys = (uint64_t)ctx->live_by_suite[QPP_SUITE_TLS_AES_128_GCM_SHA256] +
                              ctx->live_by_suite[QPP_SUITE_TLS_AES_256_GCM_SHA384];
    const uint64_t per_key = aes_keys <= kPowSlots ? kWaveKernelPacketsPerKey : kWaveKernelPacketsPerKeyNoPow;
    return (uint64_t)n < per_key * aes_keys ? AesPath::wave : AesPath::quad;
}
uint32_t aes_per_item(const qpp_ctx *ctx, AesPath p, uint32_t n) {
    return p == AesPath::burst ? burst_packets_per_item(n, ctx->n_cu)
           : p == AesPath::wave ? kWavePacketsPerItem
                                : kQuadPerItem;
}
hipError_t launch_aes(const qpp_ctx *ctx, AesPath p, bool seal, const qpp_pkt *descs, const PlanBuffers &pb, uint32_t n,
                      uint8_t *arena, uint8_t *masks, int8_t *status, uint32_t flags, hipStream_t s) {
    const uint32_t per = aes_per_item(ctx, p, n);
    switch (p) {
        case AesPath::burst:
            return launch_aes_gcm_burst(seal, ctx->d_keys, descs, pb, n, ctx->key_cap, per, arena, masks, status, flags,
                                        suite_mask(ctx), ctx->pow, s);
        case AesPath::wave:
            return launch_aes_gcm_wave(seal, ctx->d_keys, descs, pb, n, ctx->key_cap, cu_avail(ctx), arena, masks, status,
                                       flags, suite_mask(ctx), s);
        default:
            return launch_aes_gcm(seal, ctx->d_keys, descs, pb, n, cu_avail(ctx), arena, masks, status, flags,
                                  suite_mask(ctx), ctx->pow, s);
    }
}

// The one live packet key of the context when there is exactly one and it is an AES key: then a lane-kernel batch
// needs no plan (every AES packet is that key's; any other slot is refused in the kernel), saving the three plan
// launches (~25 us per 1 Mi batch).
uint32_t single_aes_slot(const qpp_ctx *ctx) {
    const uint32_t live = ctx->live_by_suite[1] + ctx->live_by_suite[2] + ctx->live_by_suite[3];
    if (live != 1 || ctx->live_by_suite[QPP_SUITE_TLS_CHACHA20_POLY1305_SHA256]) return UINT32_MAX;
    const uint32_t slot = ctx->live_slot_xor;
    return slot < ctx->key_cap && ctx->h_keys[slot].live == 1 ? slot : UINT32_MAX;
}

// Batch bodies: plan (AES) + kernels on st's stream; keys already flushed.
// The ChaCha20 kernel of a batch: after a plan that listed the non-AES packets (ChaCha20 keys, refused slots) it visits
// only those (selection mode) -- on the stream's side stream when ChaCha20 keys are live (a mixed-suite batch: it runs
// beside the AES kernel, forked behind the plan, joined before the batch ends); otherwise every packet (AES ones are
// skipped by each lane).  fork: recorded on st->stream right after the plan (the AES kernel follows it there).
hipError_t launch_chacha_batch(const qpp_ctx *ctx, StreamState *st, bool seal, bool planned, bool forked,
                               const qpp_pkt *descs, uint32_t n, uint8_t *arena, uint8_t *masks, int8_t *status,
                               uint32_t flags) {
    const bool burst = n <= (ctx->burst_max >> kChachaBurstShift);
    if (planned && !burst && plan_lists_others(n, ctx->key_cap)) {
        hipStream_t s = forked ? st->side : st->stream;
        hipError_t e = launch_chacha_sel_batch(seal, ctx->d_keys, ctx->key_cap, descs, n, arena, masks, status, flags,
                                               st->plan.perm, st->plan.n_work + 4, s);
        if (e != hipSuccess || !forked) return e;
        e = hipEventRecord(st->join_ev, st->side);
        return e != hipSuccess ? e : hipStreamWaitEvent(st->stream, st->join_ev, 0);
    }
    return launch_chacha(seal, ctx->d_keys, ctx->key_cap, descs, n, arena, masks, status, flags, burst, st->stream);
}

// Whether a planned batch forks its ChaCha20 kernel onto the side stream (ChaCha20 keys live beside AES ones, a plan
// that lists them, the lane kernel): creates the side stream on first use and records the fork point
int chacha_fork(qpp_ctx *ctx, StreamState *st, uint32_t n, uint32_t flags, bool *forked) {
    *forked = false;
    if ((flags & QPP_ONLY_AES) || !ctx->live_by_suite[QPP_SUITE_TLS_CHACHA20_POLY1305_SHA256]) return QPP_OK;
    if (n <= (ctx->burst_max >> kChachaBurstShift) || !plan_lists_others(n, ctx->key_cap)) return QPP_OK;
    static const bool off = [] {
        const char *e = getenv("QPP_CHACHA_SIDE");
        return e && e[0] == '0';
    }();
    if (off) return QPP_OK;
    if (!st->side) {
        HIP_TRY(ctx, hipStreamCreateWithFlags(&st->side, hipStreamNonBlocking));
        HIP_TRY(ctx, hipEventCreateWithFlags(&st->fork_ev, hipEventDisableTiming));
        HIP_TRY(ctx, hipEventCreateWithFlags(&st->join_ev, hipEventDisableTiming));
    }
    HIP_TRY(ctx, hipEventRecord(st->fork_ev, st->stream));
    HIP_TRY(ctx, hipStreamWaitEvent(st->side, st->fork_ev, 0));
    *forked = true;
    return QPP_OK;
}

int enqueue_seal(qpp_ctx *ctx, StreamState *st, const qpp_pkt *descs, uint32_t n, uint8_t *arena, uint8_t *masks,
                 int8_t *status, uint32_t flags, uint32_t *refused = nullptr) {
    hipStream_t s = st->stream;
    bool planned = false, forked = false;
    if (!(flags & QPP_ONLY_CHACHA)) RC_TRY(fips_gate(ctx, st, descs, n, status, refused));
    if (!(flags & QPP_ONLY_CHACHA) && (suite_mask(ctx) & kAesSuites)) {
        const AesPath path = aes_path(ctx, n);
        const uint32_t one = path == AesPath::quad ? single_aes_slot(ctx) : UINT32_MAX;
        if (one != UINT32_MAX) {
            HIP_TRY(ctx, launch_aes_gcm_single(true, ctx->d_keys, descs, one, ctx->h_keys[one].nr, n, cu_avail(ctx), arena,
                                               masks, status, flags, ctx->pow, s));
        } else {
            RC_TRY(ensure_plan(ctx, st, n));
            HIP_TRY(ctx, launch_plan(ctx->d_keys, ctx->key_cap, descs, n, st->plan, aes_per_item(ctx, path, n), s));
            RC_TRY(chacha_fork(ctx, st, n, flags, &forked));
            HIP_TRY(ctx, launch_aes(ctx, path, true, descs, st->plan, n, arena, masks, status, flags, s));
            planned = true;
        }
    }
    if (!(flags & QPP_ONLY_AES))
        HIP_TRY(ctx, launch_chacha_batch(ctx, st, true, planned, forked, descs, n, arena, masks, status, flags));
    return QPP_OK;
}

int enqueue_open(qpp_ctx *ctx, StreamState *st, const qpp_pkt *descs, uint32_t n, uint8_t *arena, int8_t *status,
                 uint32_t flags) {
    hipStream_t s = st->stream;
    bool planned = false, forked = false;
    if (!(flags & QPP_ONLY_CHACHA) && (suite_mask(ctx) & kAesSuites)) {
        const AesPath path = aes_path(ctx, n);
        const uint32_t one = path == AesPath::quad ? single_aes_slot(ctx) : UINT32_MAX;
        if (one != UINT32_MAX) {
            HIP_TRY(ctx, launch_aes_gcm_single(false, ctx->d_keys, descs, one, ctx->h_keys[one].nr, n, cu_avail(ctx), arena,
                                               nullptr, status, 0, ctx->pow, s));
        } else {
            RC_TRY(ensure_plan(ctx, st, n));
            HIP_TRY(ctx, launch_plan(ctx->d_keys, ctx->key_cap, descs, n, st->plan, aes_per_item(ctx, path, n), s));
            RC_TRY(chacha_fork(ctx, st, n, flags, &forked));
            HIP_TRY(ctx, launch_aes(ctx, path, false, descs, st->plan, n, arena, nullptr, status, 0, s));
            planned = true;
        }
    }
    if (!(flags & QPP_ONLY_AES))
        HIP_TRY(ctx, launch_chacha_batch(ctx, st, false, planned, forked, descs, n, arena, nullptr, status, 0));
    return QPP_OK;
}

// One packet through the batch kernels, zero-copy: the kernel reads and writes the pinned stage directly (no DMA
// copies; one launch, one wait).  Stage layout: descriptor @0 | perm @32 | plan meta @36 (4 words) | work item @52
// | status @72 | mask @80 | packet @kOnePkt = [pad 16 | header | payload | tag].
constexpr size_t kOnePkt = 128;
int run_one(const qpp_key *k, bool seal, uint64_t pn, const uint8_t *header, size_t header_len, const uint8_t *payload,
            size_t payload_len, uint8_t *out, uint8_t *tag_out, int8_t *status_out) {
    qpp_ctx *ctx = k->ctx;
    if (header_len > 0xffff || payload_len > 0xffff) return QPP_INTERNAL_ERROR;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    bool handled = false;
    RC_TRY(packet_server_run(k, seal, pn, header, header_len, payload, payload_len, out, tag_out, status_out, &handled));
    if (handled) return QPP_OK;
    const size_t total = kOnePkt + 16 + header_len + payload_len + 16;
    RC_TRY(ensure_stage(ctx, total));
    RC_TRY(flush_keys(ctx));
    StreamState *st = nullptr;
    RC_TRY(batch_stream(ctx, nullptr, &st));
    uint8_t *h = ctx->h_stage, *v = ctx->v_stage;
    memset(h, 0, total);
    uint8_t *pkt = h + kOnePkt;
    memcpy(pkt + 16, header, header_len);
    memcpy(pkt + 16 + header_len, payload, payload_len);
    if (!seal) memcpy(pkt + 16 + header_len + payload_len, tag_out, 16);
    qpp_pkt &d = *(qpp_pkt *)h;
    d.pn = pn;
    d.key_idx = k->slot;
    d.off = 16;
    d.aad_len = (uint16_t)header_len;
    d.pt_len = (uint16_t)payload_len;
    const uint32_t nr = ctx->h_keys[k->slot].nr;
    *(uint32_t *)(h + 32) = 0;  // perm = {0}
    uint32_t *meta = (uint32_t *)(h + 36);  // one work item, on this key, in its AES size's class
    meta[0] = 1;
    meta[1] = nr == 10 ? 1 : 0;
    meta[2] = nr == 10 ? 1 : 0;
    meta[3] = nr == 10 ? 0 : 1;
    *(WorkItem *)(h + 52) = WorkItem{k->slot, 0, 1, nr};
    h[72] = (uint8_t)QPP_INTERNAL_ERROR;  // overwritten by the kernel
    PlanBuffers pb{};
    pb.perm = (uint32_t *)(v + 32);
    pb.work = (WorkItem *)(v + 52);
    pb.n_work = (uint32_t *)(v + 36);
    hipStream_t s = ctx->stream;
    const qpp_pkt *vd = (const qpp_pkt *)v;
    int8_t *vst = (int8_t *)(v + 72);
    if (seal && ctx->h_keys[k->slot].fips) {  // FIPS mode: the nonce-order gate (refused: status INTERNAL_ERROR)
        RC_TRY(fips_gate(ctx, st, vd, 1, vst, nullptr));
    }
    if (is_aes(k->suite)) {
        // key_cap = 0: grid = plan_max_work(1, 0, per) = 1; only work item 0 exists
        if (ctx->burst_max)
            HIP_TRY(ctx, launch_aes_gcm_burst(seal, ctx->d_keys, vd, pb, 1, 0, 1, v + kOnePkt, v + 80, vst, 0,
                                              1u << k->suite, ctx->pow, s));
        else
            HIP_TRY(ctx, launch_aes_gcm(seal, ctx->d_keys, vd, pb, 1, 1, v + kOnePkt, v + 80, vst, 0, 1u << k->suite,
                                        ctx->pow, s));
    } else {
        HIP_TRY(ctx, launch_chacha(seal, ctx->d_keys, ctx->key_cap, vd, 1, v + kOnePkt, v + 80, vst, 0,
                                   ctx->burst_max > 0, s));
    }
    RC_TRY(note_work(ctx, st));
    HIP_TRY(ctx, hipStreamSynchronize(s));
    *status_out = (int8_t)h[72];
    if (seal && *status_out != QPP_OK) {  // refused (FIPS nonce order): the caller's buffer stays untouched
        secure_zero(h, total);
        return QPP_OK;
    }
    memcpy(out, pkt + 16 + header_len, payload_len);
    if (seal) memcpy(tag_out, pkt + 16 + header_len + payload_len, 16);
    secure_zero(h, total);
    return QPP_OK;
}

// HeaderKey::*_header_protection_mask for one sample through the hp_mask kernel, zero-copy on the pinned stage:
// descriptor @0, sample @64 (+4), mask @96.
int mask_one(qpp_ctx *ctx, uint32_t slot, const uint8_t *sample, uint8_t mask[5]) {
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    bool handled = false;
    RC_TRY(packet_server_mask(ctx, slot, sample, mask, &handled));
    if (handled) return QPP_OK;
    RC_TRY(ensure_stage(ctx, 128));
    RC_TRY(flush_keys(ctx));
    StreamState *st = nullptr;
    RC_TRY(batch_stream(ctx, nullptr, &st));
    uint8_t *h = ctx->h_stage;
    memset(h, 0, 128);
    memcpy(h + 64 + 4, sample, 16);
    qpp_pkt &d = *(qpp_pkt *)h;
    d.key_idx = slot;  // off = aad_len = pn_len = 0: sample at offset 4
    hipStream_t s = ctx->stream;
    HIP_TRY(ctx, launch_hp_mask(ctx->d_keys, ctx->key_cap, (const qpp_pkt *)ctx->v_stage, 1, ctx->v_stage + 64,
                                ctx->v_stage + 96, s));
    RC_TRY(note_work(ctx, st));
    HIP_TRY(ctx, hipStreamSynchronize(s));
    memcpy(mask, h + 96, 5);
    return QPP_OK;
}

int derive_batch_device(qpp_ctx *ctx, int suite, const uint8_t *secrets, const uint8_t *hp_in, size_t n,
                        uint32_t updates, const std::vector<uint32_t> &slots, qpp_key **out);

// n secrets (n * hash_len, host) [+ header keys hp_in, n * key_len, host] -> n device-derived keys in fresh or
// recycled slots.  updates x "quic ku" on each; material copied back for the host handles.
int derive_batch(qpp_ctx *ctx, int suite, const uint8_t *secrets, const uint8_t *hp_in, size_t n, uint32_t updates,
                 qpp_key **out) {
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    RC_TRY(flush_keys(ctx));  // pending host records first
    // (The records that flush just queued are copied from its key stage asynchronously; the derivation takes the
    // OTHER stage -- take_kstage -- so it neither waits for that copy nor overwrites the records: overwriting them was
    // found by tests/test_gpu_fuzz.py, a key created just before a batched update installed from the secrets written
    // over its record.)
    std::vector<uint32_t> slots;
    slots.reserve(n);
    // a failure after slots were taken gives them back through retirement (the device may have written their records)
    auto give_back = [&](int rc) {
        for (uint32_t s : slots) retire_slot(ctx, s);
        return rc;
    };
    for (size_t i = 0; i < n; i++) {
        uint32_t s = 0;
        if (int rc = alloc_slot(ctx, &s)) return give_back(rc);
        slots.push_back(s);
    }
    if (int rc = derive_batch_device(ctx, suite, secrets, hp_in, n, updates, slots, out)) return give_back(rc);
    return QPP_OK;
}

// derive_batch after the slots are taken: stage, derive on the device, copy the material back, make the handles
int derive_batch_device(qpp_ctx *ctx, int suite, const uint8_t *secrets, const uint8_t *hp_in, size_t n,
                        uint32_t updates, const std::vector<uint32_t> &slots, qpp_key **out) {
    const size_t hl = suite_hash_len(suite), kl = suite_key_len(suite), mb = key_material_bytes();
    // key stage: secrets | hp_in | slots | material
    const size_t o_hp = n * hl, o_slot = o_hp + (hp_in ? n * kl : 0), o_mat = (o_slot + 4 * n + 15) & ~size_t(15);
    const size_t total = o_mat + n * mb;
    KStage *ks = nullptr;
    RC_TRY(take_kstage(ctx, total, &ks));
    uint8_t *h = ks->h, *d = ks->d;
    // the pinned stage holds secrets from here on: any exit below leaves them to the next take_kstage to zeroize
    ks->pending = total;
    memcpy(h, secrets, n * hl);
    if (hp_in) memcpy(h + o_hp, hp_in, n * kl);
    memcpy(h + o_slot, slots.data(), 4 * n);
    hipStream_t s = ctx->kstream;
    HIP_TRY(ctx, hipMemcpyAsync(d, h, o_slot + 4 * n, hipMemcpyHostToDevice, s));
    HIP_TRY(ctx, launch_key_derive(ctx->d_keys, (const uint32_t *)(d + o_slot), (uint32_t)n, suite, d,
                                   hp_in ? d + o_hp : nullptr, updates, d + o_mat, ctx->fips ? 1u : 0u, ctx->pow, s));
    HIP_TRY(ctx, hipMemcpyAsync(h + o_mat, d + o_mat, n * mb, hipMemcpyDeviceToHost, s));
    HIP_TRY(ctx, hipMemsetAsync(d, 0, total, s));
    HIP_TRY(ctx, hipEventRecord(ctx->keys_ready, s));
    ctx->key_gen++;
    RC_TRY(release_kstage(ctx, ks, total));  // (zeroized below as well; an error exit in between leaves it pending)
    HIP_TRY(ctx, hipStreamSynchronize(s));  // the material comes back to the host handles
    const uint32_t nr = suite == QPP_SUITE_TLS_AES_128_GCM_SHA256 ? 10 : suite == QPP_SUITE_TLS_AES_256_GCM_SHA384 ? 14 : 0;
    for (size_t i = 0; i < n; i++) {
        const uint8_t *m = h + o_mat + i * mb;
        qpp_key *k = new qpp_key();
        k->ctx = ctx;
        k->suite = suite;
        k->slot = slots[i];
        k->has_secret = true;
        memcpy(k->secret, m, hl);
        memcpy(k->key, m + 48, kl);
        memcpy(k->iv, m + 80, 12);
        memcpy(k->hp, m + 96, kl);
        // host mirror: what the host needs (suite, rounds, liveness); the record itself was written on the device
        DevKey &r = ctx->h_keys[slots[i]];
        memset(&r, 0, sizeof r);
        r.suite = (uint32_t)suite;
        r.nr = r.hp_nr = nr;
        r.live = 1;
        r.fips = ctx->fips && is_aes(suite) ? 1u : 0u;  // as key_derive_kernel sets it on the device
        ctx->fips_live += r.fips;
        ctx->live_slot_xor ^= slots[i];
        out[i] = k;
    }
    ctx->live_by_suite[suite] += (uint32_t)n;
    secure_zero(h, total);
    return QPP_OK;
}

// ---------------------------------------------------------------- host pipeline

int pipe_init(qpp_ctx *ctx) {
    HostPipe *p = ctx->pipe;
    if (!p->h2d) {
        HIP_TRY(ctx, hipStreamCreateWithFlags(&p->h2d, hipStreamNonBlocking));
        HIP_TRY(ctx, hipStreamCreateWithFlags(&p->comp, hipStreamNonBlocking));
        HIP_TRY(ctx, hipStreamCreateWithFlags(&p->d2h, hipStreamNonBlocking));
    }
    if (p->slots.size() == p->nslots && !p->slots.empty() && p->slots[0].arena) return QPP_OK;
    p->slots.resize(p->nslots);
    for (PipeSlot &sl : p->slots) {
        HIP_TRY(ctx, dmalloc(ctx, &sl.arena, p->chunk_bytes));
        HIP_TRY(ctx, dmalloc(ctx, &sl.descs, sizeof(qpp_pkt) * p->chunk_packets));
        HIP_TRY(ctx, dmalloc(ctx, &sl.masks, 5 * p->chunk_packets));
        HIP_TRY(ctx, dmalloc(ctx, &sl.status, p->chunk_packets));
        HIP_TRY(ctx, hipEventCreateWithFlags(&sl.h2d, hipEventDisableTiming));
        HIP_TRY(ctx, hipEventCreateWithFlags(&sl.comp, hipEventDisableTiming));
        HIP_TRY(ctx, hipEventCreateWithFlags(&sl.d2h, hipEventDisableTiming));
        sl.busy = false;
    }
    p->next = 0;
    return QPP_OK;
}

void pipe_release(qpp_ctx *ctx) {
    HostPipe *p = ctx->pipe;
    if (!p) return;
    for (hipStream_t s : {p->h2d, p->comp, p->d2h})
        if (s) hipStreamSynchronize(s);  // no chunk is in flight
    for (PipeSlot &sl : p->slots) {
        if (sl.arena) {
            hipMemsetAsync(sl.arena, 0, p->chunk_bytes, ctx->stream);
            hipStreamSynchronize(ctx->stream);
            dfree(ctx, sl.arena);
        }
        dfree(ctx, sl.descs); dfree(ctx, sl.masks); dfree(ctx, sl.status);
        if (sl.h2d) hipEventDestroy(sl.h2d);
        if (sl.comp) hipEventDestroy(sl.comp);
        if (sl.d2h) hipEventDestroy(sl.d2h);
        sl = PipeSlot{};
    }
    p->slots.clear();
}

}  // namespace

extern "C" {

int qpp_abi_version(void) { return QPP_ABI_VERSION; }

int qpp_ctx_create(int device, qpp_ctx **out) {
    if (!out) return QPP_INTERNAL_ERROR;
    *out = nullptr;
    int count = 0;
    if (hipGetDeviceCount(&count) != hipSuccess || device < 0 || device >= count) return QPP_DEVICE_ERROR;
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess) return QPP_DEVICE_ERROR;
    if (strncmp(prop.gcnArchName, "gfx950", 6) != 0) return QPP_DEVICE_ERROR;  // kernels are built for gfx950 only
    qpp_ctx *ctx = new qpp_ctx();
    ctx->device = device;
    ctx->n_cu = (uint32_t)prop.multiProcessorCount;
    if (const char *e = getenv("QPP_BURST_MAX")) ctx->burst_max = (uint32_t)strtoul(e, nullptr, 10);
    if (const char *e = getenv("QPP_PACKET_SERVER")) ctx->pkt_server = strcmp(e, "0") != 0;
    if (const char *e = getenv("QPP_AES_KERNEL"))
        ctx->aes_kernel = !strcmp(e, "quad") || !strcmp(e, "lane") ? QPP_AES_KERNEL_QUAD
                        : !strcmp(e, "wave")                     ? QPP_AES_KERNEL_WAVE
                                                                 : 0;
    int rc = QPP_OK;
    do {
        if (fail(ctx, hipSetDevice(device), "hipSetDevice")) { rc = QPP_DEVICE_ERROR; break; }
        if (fail(ctx, hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking), "stream") ||
            fail(ctx, hipStreamCreateWithFlags(&ctx->kstream, hipStreamNonBlocking), "key stream") ||
            fail(ctx, hipStreamCreateWithFlags(&ctx->rstream, hipStreamNonBlocking), "retire stream") ||
            fail(ctx, hipEventCreateWithFlags(&ctx->keys_ready, hipEventDisableTiming), "key event")) {
            rc = QPP_DEVICE_ERROR;
            break;
        }
        if (!stream_state(ctx, ctx->stream)) { rc = QPP_DEVICE_ERROR; break; }
        if (fail(ctx, dmalloc(ctx, &ctx->d_diag, 64), "diag") ||
            fail(ctx, hipMemsetAsync(ctx->d_diag, 0, 64, ctx->stream), "diag") ||
            fail(ctx, hipStreamSynchronize(ctx->stream), "diag")) {
            rc = QPP_DEVICE_ERROR;
            break;
        }
        rc = grow_keys(ctx, 64);
    } while (0);
    if (rc) {
        qpp_ctx_destroy(ctx);
        return rc;
    }
    *out = ctx;
    return QPP_OK;
}

int qpp_ctx_set_aes_kernel(qpp_ctx *ctx, int kernel) {
    if (!ctx || kernel < QPP_AES_KERNEL_AUTO || kernel > QPP_AES_KERNEL_WAVE) return QPP_INTERNAL_ERROR;
    ctx->aes_kernel = kernel;
    return QPP_OK;
}

int qpp_ctx_set_fips(qpp_ctx *ctx, int on) {
    if (!ctx) return QPP_INTERNAL_ERROR;
    ctx->fips = on != 0;
    return QPP_OK;
}

int qpp_key_fips(const qpp_key *key) {
    if (!key || !key->ctx || key->slot >= key->ctx->key_cap) return 0;
    return key->ctx->h_keys[key->slot].fips ? 1 : 0;
}

int qpp_ctx_set_burst_max(qpp_ctx *ctx, size_t max_packets) {
    if (!ctx) return QPP_INTERNAL_ERROR;
    ctx->burst_max = max_packets > UINT32_MAX ? UINT32_MAX : (uint32_t)max_packets;
    return QPP_OK;
}

void qpp_ctx_destroy(qpp_ctx *ctx) {
    if (!ctx) return;
    hipSetDevice(ctx->device);
    qpp_txq_destroy(ctx->pkt_q);
    ctx->pkt_q = nullptr;
    if (ctx->d_keys) flush_retire(ctx);  // pending zeroizations, while the table and the stream states still exist
    servers_stop(ctx);
    ctx_sync(ctx);  // (the context's streams only: another context's resident servers may run on)
    if (ctx->d_keys) {
        hipMemsetAsync(ctx->d_keys, 0, sizeof(DevKey) * ctx->key_cap, ctx->stream);
        hipStreamSynchronize(ctx->stream);
        dfree(ctx, ctx->d_keys);
    }
    secure_zero(ctx->h_keys.data(), sizeof(DevKey) * ctx->h_keys.size());
    if (ctx->pow.base) {
        hipMemsetAsync(ctx->pow.base, 0, (size_t)ctx->pow.cap * kPowBytes, ctx->stream);
        hipStreamSynchronize(ctx->stream);
        dfree(ctx, ctx->pow.base);
    }
    for (StreamState *st : ctx->streams) free_stream_state(ctx, st);
    ctx->streams.clear();
    for (Retired &r : ctx->retired) hipEventDestroy(r.done);
    for (hipEvent_t e : ctx->event_pool) hipEventDestroy(e);
    if (ctx->pipe) {
        pipe_release(ctx);
        for (auto &t : ctx->pipe->tickets) hipEventDestroy(t.second);
        if (ctx->pipe->h2d) hipStreamDestroy(ctx->pipe->h2d);
        if (ctx->pipe->comp) hipStreamDestroy(ctx->pipe->comp);
        if (ctx->pipe->d2h) hipStreamDestroy(ctx->pipe->d2h);
        delete ctx->pipe;
    }
    dfree(ctx, ctx->d_stage);
    dfree(ctx, ctx->d_connmap);
    dfree(ctx, ctx->d_diag);
    hfree(ctx, ctx->h_connstage);
    if (ctx->connstage_ev) hipEventDestroy(ctx->connstage_ev);
    hfree(ctx, ctx->h_stage);
    for (KStage &k : ctx->kstage) {
        dfree(ctx, k.d);
        if (k.h) { secure_zero(k.h, k.cap); hfree(ctx, k.h); }
        if (k.free_ev) hipEventDestroy(k.free_ev);
    }
    if (ctx->stream) hipStreamDestroy(ctx->stream);
    if (ctx->kstream) hipStreamDestroy(ctx->kstream);
    if (ctx->rstream) hipStreamDestroy(ctx->rstream);
    if (ctx->keys_ready) hipEventDestroy(ctx->keys_ready);
    if (ctx->fips_order) hipEventDestroy(ctx->fips_order);
    delete ctx;
}

void *qpp_ctx_stream(qpp_ctx *ctx) { return ctx ? (void *)ctx->stream : nullptr; }

int qpp_ctx_synchronize(qpp_ctx *ctx) {
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    RC_TRY(flush_retire(ctx));
    RC_TRY(servers_stop(ctx));  // (restarted by the next flush of their queue)
    RC_TRY(ctx_sync(ctx));      // every stream of the context (not the device: other contexts' servers run on)
    hfree(ctx, nullptr);        // pinned buffers parked while other contexts' servers were resident
    return QPP_OK;
}

const char *qpp_ctx_last_error(qpp_ctx *ctx) { return ctx ? ctx->last_error.c_str() : "no context"; }

int qpp_ctx_rx_timeouts(qpp_ctx *ctx, uint64_t *count) {
    if (!ctx || !count) return QPP_INTERNAL_ERROR;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    for (StreamState *st : ctx->streams) HIP_TRY(ctx, hipStreamSynchronize(st->stream));
    uint32_t v = 0;
    HIP_TRY(ctx, hipMemcpyAsync(&v, ctx->d_diag, 4, hipMemcpyDeviceToHost, ctx->stream));
    HIP_TRY(ctx, hipStreamSynchronize(ctx->stream));
    *count = v;
    return QPP_OK;
}

int qpp_ctx_key_slots(qpp_ctx *ctx, uint32_t *capacity, uint32_t *high_water, uint32_t *retired) {
    if (!ctx) return QPP_INTERNAL_ERROR;
    if (capacity) *capacity = ctx->key_cap;
    if (high_water) *high_water = ctx->next_slot;
    if (retired) *retired = ctx->retired_slots + (uint32_t)ctx->retire_pending.size();
    return QPP_OK;
}

// ---------------------------------------------------------------- keys

int qpp_key_new(qpp_ctx *ctx, int suite, const uint8_t *secret, size_t secret_len, qpp_key **out) {
    if (!ctx || !out || !secret) return QPP_INTERNAL_ERROR;
    *out = nullptr;
    if (!valid_suite(suite)) return QPP_UNSUPPORTED;
    if (secret_len != suite_hash_len(suite)) return QPP_INTERNAL_ERROR;
    qpp_key *k = new qpp_key();
    k->ctx = ctx;
    k->suite = suite;
    k->has_secret = true;
    memcpy(k->secret, secret, secret_len);
    derive(k);
    int rc = install(k);
    if (rc) { secure_zero(k, sizeof *k); delete k; return rc; }
    *out = k;
    return QPP_OK;
}

int qpp_key_new_pair(qpp_ctx *ctx, int suite, const uint8_t *secret, size_t secret_len, qpp_key **key,
                     qpp_header_key **header_key) {
    if (!key || !header_key) return QPP_INTERNAL_ERROR;
    *header_key = nullptr;
    RC_TRY(qpp_key_new(ctx, suite, secret, secret_len, key));
    int rc = qpp_header_key_new(ctx, suite, secret, secret_len, header_key);
    if (rc) { qpp_key_free(*key); *key = nullptr; }
    return rc;
}

int qpp_key_new_batch(qpp_ctx *ctx, int suite, const uint8_t *secrets, size_t n, uint32_t updates, qpp_key **out) {
    if (!ctx || !out || (n && !secrets)) return QPP_INTERNAL_ERROR;
    if (!valid_suite(suite)) return QPP_UNSUPPORTED;
    if (n > (1u << 24)) return QPP_INTERNAL_ERROR;
    if (!n) return QPP_OK;
    return derive_batch(ctx, suite, secrets, nullptr, n, updates, out);
}

int qpp_key_update_batch(qpp_key *const *keys, size_t n, qpp_key **out) {
    if (!out || (n && !keys)) return QPP_INTERNAL_ERROR;
    if (!n) return QPP_OK;
    if (n > (1u << 24)) return QPP_INTERNAL_ERROR;
    for (size_t i = 0; i < n; i++) out[i] = nullptr;  // the caller's array may be uninitialised
    qpp_ctx *ctx = keys[0] ? keys[0]->ctx : nullptr;
    if (!ctx) return QPP_INTERNAL_ERROR;
    for (size_t i = 0; i < n; i++)
        if (!keys[i] || keys[i]->ctx != ctx || !keys[i]->has_secret) return QPP_INTERNAL_ERROR;
    // one device pass per suite present, each key's secret through one "quic ku" step, its header key kept
    std::vector<uint8_t> sec, hp;
    std::vector<size_t> idx;
    std::vector<qpp_key *> made;
    for (int suite = 1; suite <= 3; suite++) {
        idx.clear();
        for (size_t i = 0; i < n; i++)
            if (keys[i]->suite == suite) idx.push_back(i);
        if (idx.empty()) continue;
        const size_t hl = suite_hash_len(suite), kl = suite_key_len(suite);
        sec.resize(idx.size() * hl);
        hp.resize(idx.size() * kl);
        for (size_t j = 0; j < idx.size(); j++) {
            memcpy(sec.data() + j * hl, keys[idx[j]]->secret, hl);
            memcpy(hp.data() + j * kl, keys[idx[j]]->hp, kl);
        }
        made.resize(idx.size());
        int rc = derive_batch(ctx, suite, sec.data(), hp.data(), idx.size(), 1, made.data());
        secure_zero(sec.data(), sec.size());
        secure_zero(hp.data(), hp.size());
        if (rc) {
            for (size_t i = 0; i < n; i++)
                if (out[i]) { qpp_key_free(out[i]); out[i] = nullptr; }
            return rc;
        }
        for (size_t j = 0; j < idx.size(); j++) out[idx[j]] = made[j];
    }
    return QPP_OK;
}

int qpp_key_new_raw(qpp_ctx *ctx, int suite, const uint8_t *key, size_t key_len, const uint8_t iv[12],
                    const uint8_t *hp, size_t hp_len, qpp_key **out) {
    if (!ctx || !out || !key || !iv || !hp) return QPP_INTERNAL_ERROR;
    *out = nullptr;
    if (!valid_suite(suite)) return QPP_UNSUPPORTED;
    if (key_len != suite_key_len(suite) || hp_len != suite_key_len(suite)) return QPP_INTERNAL_ERROR;
    qpp_key *k = new qpp_key();
    k->ctx = ctx;
    k->suite = suite;
    memcpy(k->key, key, key_len);
    memcpy(k->iv, iv, 12);
    memcpy(k->hp, hp, hp_len);
    int rc = install(k);
    if (rc) { secure_zero(k, sizeof *k); delete k; return rc; }
    *out = k;
    return QPP_OK;
}

int qpp_key_update(const qpp_key *key, qpp_key **out) {
    if (!key || !out) return QPP_INTERNAL_ERROR;
    *out = nullptr;
    if (!key->has_secret) return QPP_INTERNAL_ERROR;
    qpp_key *k = new qpp_key();
    k->ctx = key->ctx;
    k->suite = key->suite;
    k->has_secret = true;
    const size_t hl = suite_hash_len(key->suite);
    hkdf_expand_label(hl, key->secret, "quic ku", k->secret, hl);
    derive(k);
    memcpy(k->hp, key->hp, sizeof k->hp);  // RFC 9001 §6: the header protection key is not updated
    int rc = install(k);
    if (rc) { secure_zero(k, sizeof *k); delete k; return rc; }
    *out = k;
    return QPP_OK;
}

void qpp_key_free(qpp_key *key) {
    if (!key) return;
    qpp_ctx *ctx = key->ctx;
    if (ctx && key->slot < ctx->key_cap && ctx->h_keys[key->slot].live == 1) {
        ctx->live_by_suite[key->suite]--;
        ctx->live_slot_xor ^= key->slot;
        ctx->fips_live -= ctx->h_keys[key->slot].fips;
        retire_slot(ctx, key->slot);
    }
    secure_zero(key, sizeof *key);
    delete key;
}

void qpp_key_free_batch(qpp_key *const *keys, size_t n) {
    if (!keys) return;
    for (size_t i = 0; i < n; i++) qpp_key_free(keys[i]);  // retirements only collect; one flush before the next use
}

uint32_t qpp_key_slot(const qpp_key *key) { return key ? key->slot : UINT32_MAX; }
void qpp_key_slot_batch(const qpp_key *const *keys, size_t n, uint32_t *slots) {
    if (!keys || !slots) return;
    for (size_t i = 0; i < n; i++) slots[i] = keys[i] ? keys[i]->slot : UINT32_MAX;
}
int qpp_key_suite(const qpp_key *key) { return key ? key->suite : 0; }
size_t qpp_tag_len(const qpp_key *) { return 16; }
size_t qpp_sample_len(const qpp_key *) { return 16; }
uint64_t qpp_confidentiality_limit(const qpp_key *key) {
    // cipher_suite.rs:261,281,298 (RFC 9001 §6.6)
    return key && key->suite == QPP_SUITE_TLS_CHACHA20_POLY1305_SHA256 ? (1ULL << 62) : (1ULL << 23);
}
uint64_t qpp_integrity_limit(const qpp_key *key) {
    // cipher_suite.rs:262,282,299
    return key && key->suite == QPP_SUITE_TLS_CHACHA20_POLY1305_SHA256 ? (1ULL << 36) : (1ULL << 52);
}

int qpp_key_material(const qpp_key *key, uint8_t *key_out, uint8_t iv_out[12], uint8_t *hp_out) {
    if (!key) return QPP_INTERNAL_ERROR;
    const size_t kl = suite_key_len(key->suite);
    if (key_out) memcpy(key_out, key->key, kl);
    if (iv_out) memcpy(iv_out, key->iv, 12);
    if (hp_out) memcpy(hp_out, key->hp, kl);
    return QPP_OK;
}

// ---------------------------------------------------------------- header keys (header_key.rs)

int qpp_header_key_new_raw(qpp_ctx *ctx, int suite, const uint8_t *hp, size_t hp_len, qpp_header_key **out) {
    if (!ctx || !out || !hp) return QPP_INTERNAL_ERROR;
    *out = nullptr;
    if (!valid_suite(suite)) return QPP_UNSUPPORTED;
    if (hp_len != suite_key_len(suite)) return QPP_INTERNAL_ERROR;
    qpp_header_key *h = new qpp_header_key();
    h->ctx = ctx;
    h->suite = suite;
    memcpy(h->hp, hp, hp_len);
    int rc = install_header(h);
    if (rc) { secure_zero(h, sizeof *h); delete h; return rc; }
    *out = h;
    return QPP_OK;
}

int qpp_header_key_new(qpp_ctx *ctx, int suite, const uint8_t *secret, size_t secret_len, qpp_header_key **out) {
    // HeaderKey::new(secret, "quic hp", alg) (header_key.rs:33-49), as TLS_*::new makes it (cipher_suite.rs:85-103)
    if (!ctx || !out || !secret) return QPP_INTERNAL_ERROR;
    *out = nullptr;
    if (!valid_suite(suite)) return QPP_UNSUPPORTED;
    if (secret_len != suite_hash_len(suite)) return QPP_INTERNAL_ERROR;
    uint8_t hp[32];
    const size_t kl = suite_key_len(suite);
    hkdf_expand_label(secret_len, secret, "quic hp", hp, kl);
    int rc = qpp_header_key_new_raw(ctx, suite, hp, kl, out);
    secure_zero(hp, sizeof hp);
    return rc;
}

void qpp_header_key_free(qpp_header_key *hk) {
    if (!hk) return;
    qpp_ctx *ctx = hk->ctx;
    if (ctx && hk->slot < ctx->key_cap && ctx->h_keys[hk->slot].live == 2) {
        ctx->hdr_live_by_suite[ctx->h_keys[hk->slot].suite & 3]--;
        retire_slot(ctx, hk->slot);
    }
    secure_zero(hk, sizeof *hk);
    delete hk;
}

uint32_t qpp_header_key_slot(const qpp_header_key *hk) { return hk ? hk->slot : UINT32_MAX; }
int qpp_header_key_suite(const qpp_header_key *hk) { return hk ? hk->suite : 0; }
size_t qpp_header_key_sample_len(const qpp_header_key *) { return 16; }

int qpp_header_key_mask(const qpp_header_key *hk, const uint8_t *sample, size_t sample_len, uint8_t mask[5]) {
    if (!hk || !sample || !mask || sample_len < 16) return QPP_INTERNAL_ERROR;
    return mask_one(hk->ctx, hk->slot, sample, mask);
}

int qpp_initial_keys(qpp_ctx *ctx, int endpoint, const uint8_t *dcid, size_t dcid_len, qpp_key **sealer,
                     qpp_key **opener) {
    return qpp_initial_keys_pair(ctx, endpoint, dcid, dcid_len, sealer, opener, nullptr, nullptr);
}

int qpp_initial_keys_pair(qpp_ctx *ctx, int endpoint, const uint8_t *dcid, size_t dcid_len, qpp_key **sealer,
                          qpp_key **opener, qpp_header_key **header_sealer, qpp_header_key **header_opener) {
    // quic/s2n-quic-crypto/src/initial.rs:29-68 -> (InitialKey, InitialHeaderKey); salt quic/s2n-quic-core/src/crypto/initial.rs:29
    static const uint8_t salt[20] = {0x38, 0x76, 0x2c, 0xf7, 0xf5, 0x59, 0x34, 0xb3, 0x4d, 0x17,
                                     0x9a, 0xe6, 0xa4, 0xc8, 0x0c, 0xad, 0xcc, 0xbb, 0x7f, 0x0a};
    if (!ctx || !sealer || !opener || (!dcid && dcid_len)) return QPP_INTERNAL_ERROR;
    if (!header_sealer != !header_opener) return QPP_INTERNAL_ERROR;
    *sealer = *opener = nullptr;
    if (header_sealer) *header_sealer = *header_opener = nullptr;
    uint8_t prk[32], client[32], server[32];
    hkdf_extract(32, salt, sizeof salt, dcid, dcid_len, prk);
    hkdf_expand_label(32, prk, "client in", client, 32);
    hkdf_expand_label(32, prk, "server in", server, 32);
    const bool is_client = endpoint == QPP_ENDPOINT_CLIENT;
    const uint8_t *ss = is_client ? client : server, *os = is_client ? server : client;
    const int suite = QPP_SUITE_TLS_AES_128_GCM_SHA256;
    int rc = qpp_key_new(ctx, suite, ss, 32, sealer);
    if (!rc) rc = qpp_key_new(ctx, suite, os, 32, opener);
    if (!rc && header_sealer) rc = qpp_header_key_new(ctx, suite, ss, 32, header_sealer);
    if (!rc && header_opener) rc = qpp_header_key_new(ctx, suite, os, 32, header_opener);
    if (rc) {
        qpp_key_free(*sealer); qpp_key_free(*opener);
        *sealer = *opener = nullptr;
        if (header_sealer) {
            qpp_header_key_free(*header_sealer); qpp_header_key_free(*header_opener);
            *header_sealer = *header_opener = nullptr;
        }
    }
    secure_zero(prk, sizeof prk); secure_zero(client, sizeof client); secure_zero(server, sizeof server);
    return rc;
}

// ---------------------------------------------------------------- per packet

int qpp_seal(qpp_key *key, uint64_t pn, const uint8_t *header, size_t header_len, uint8_t *payload, size_t payload_len,
             size_t payload_cap) {
    if (!key || (!header && header_len) || (!payload && payload_len)) return QPP_INTERNAL_ERROR;
    if (payload_cap < payload_len + 16) return QPP_INTERNAL_ERROR;
    int8_t st;
    int rc = run_one(key, true, pn, header, header_len, payload, payload_len, payload, payload + payload_len, &st);
    return rc ? rc : st;
}

int qpp_seal_scatter(qpp_key *key, uint64_t pn, const uint8_t *header, size_t header_len, uint8_t *in_out,
                     size_t in_len, const uint8_t *extra_in, size_t extra_len, uint8_t *extra_out_and_tag) {
    if (!key || (!in_out && in_len) || (!extra_in && extra_len) || !extra_out_and_tag) return QPP_INTERNAL_ERROR;
    std::vector<uint8_t> flat(in_len + extra_len);
    if (in_len) memcpy(flat.data(), in_out, in_len);
    if (extra_len) memcpy(flat.data() + in_len, extra_in, extra_len);
    int8_t st;
    int rc = run_one(key, true, pn, header, header_len, flat.data(), flat.size(), flat.data(), extra_out_and_tag + extra_len, &st);
    if (!rc) {
        if (in_len) memcpy(in_out, flat.data(), in_len);
        if (extra_len) memcpy(extra_out_and_tag, flat.data() + in_len, extra_len);
    }
    secure_zero(flat.data(), flat.size());
    return rc ? rc : st;
}

int qpp_open(const qpp_key *key, uint64_t pn, const uint8_t *header, size_t header_len, uint8_t *payload,
             size_t payload_len) {
    if (!key || (!header && header_len) || (!payload && payload_len)) return QPP_INTERNAL_ERROR;
    if (payload_len < 16) return QPP_DECRYPT_ERROR;  // cipher_suite.rs:126-129
    uint8_t tag[16];
    memcpy(tag, payload + payload_len - 16, 16);
    int8_t st;
    int rc = run_one(key, false, pn, header, header_len, payload, payload_len - 16, payload, tag, &st);
    return rc ? rc : st;
}

int qpp_hp_mask(const qpp_key *key, const uint8_t *sample, size_t sample_len, uint8_t mask[5]) {
    if (!key || !sample || !mask || sample_len < 16) return QPP_INTERNAL_ERROR;
    return mask_one(key->ctx, key->slot, sample, mask);
}

// ---------------------------------------------------------------- dc consumers (dc/s2n-quic-dc/src/crypto/awslc.rs)

int qpp_dc_key_new(qpp_ctx *ctx, int suite, const uint8_t *key, size_t key_len, const uint8_t iv[12], qpp_key **out) {
    // awslc.rs:24-33,157-166: key + iv only; the unused header-key slot stays zero
    static const uint8_t no_hp[32] = {0};
    if (!valid_suite(suite)) return QPP_UNSUPPORTED;
    return qpp_key_new_raw(ctx, suite, key, key_len, iv, no_hp, suite_key_len(suite), out);
}

int qpp_dc_seal(const qpp_key *key, uint64_t pn, const uint8_t *header, size_t header_len, const uint8_t *extra_payload,
                size_t extra_len, uint8_t *payload_and_tag, size_t len) {
    // awslc.rs:53-83: inline_len = len - tag - extra; seal_in_place_scatter(in_out = [0, inline), extra_out_and_tag)
    if (!key || (!header && header_len) || (!extra_payload && extra_len) || !payload_and_tag) return QPP_INTERNAL_ERROR;
    if (len < 16 || len - 16 < extra_len) return QPP_INTERNAL_ERROR;
    const size_t msg = len - 16, inline_len = msg - extra_len;
    int8_t st;
    int rc;
    if (!extra_len) {
        rc = run_one(key, true, pn, header, header_len, payload_and_tag, msg, payload_and_tag, payload_and_tag + msg, &st);
    } else {
        std::vector<uint8_t> flat(msg);  // inline || extra as one message; the sealed bytes land in payload_and_tag
        if (inline_len) memcpy(flat.data(), payload_and_tag, inline_len);
        memcpy(flat.data() + inline_len, extra_payload, extra_len);
        rc = run_one(key, true, pn, header, header_len, flat.data(), msg, payload_and_tag, payload_and_tag + msg, &st);
        secure_zero(flat.data(), flat.size());
    }
    return rc ? rc : st;
}

int qpp_dc_open(const qpp_key *key, int key_phase, uint64_t pn, const uint8_t *header, size_t header_len,
                const uint8_t *payload_in, const uint8_t *tag, size_t tag_len, uint8_t *payload_out, size_t payload_len) {
    // awslc.rs:176-204: ensure!(key_phase == Zero, RotationNotSupported); open_separate_gather -> InvalidTag
    if (!key || (!header && header_len) || ((!payload_in || !payload_out) && payload_len) || (!tag && tag_len))
        return QPP_INTERNAL_ERROR;
    if (key_phase != 0) return QPP_ROTATION_NOT_SUPPORTED;
    if (tag_len != 16) {
        if (payload_len) memset(payload_out, 0, payload_len);
        return QPP_DECRYPT_ERROR;
    }
    uint8_t t[16];
    memcpy(t, tag, 16);
    int8_t st;
    int rc = run_one(key, false, pn, header, header_len, payload_in, payload_len, payload_out, t, &st);
    return rc ? rc : st;
}

int qpp_dc_open_in_place(const qpp_key *key, int key_phase, uint64_t pn, const uint8_t *header, size_t header_len,
                         uint8_t *payload, size_t payload_len, const uint8_t *tag, size_t tag_len) {
    // awslc.rs:207-227: open_in_place_separate_tag
    if (!key || (!header && header_len) || (!payload && payload_len) || (!tag && tag_len)) return QPP_INTERNAL_ERROR;
    if (key_phase != 0) return QPP_ROTATION_NOT_SUPPORTED;
    if (tag_len != 16) return QPP_DECRYPT_ERROR;
    uint8_t t[16];
    memcpy(t, tag, 16);
    int8_t st;
    int rc = run_one(key, false, pn, header, header_len, payload, payload_len, payload, t, &st);
    return rc ? rc : st;
}

// ---------------------------------------------------------------- batches

int qpp_seal_batch(qpp_ctx *ctx, const qpp_pkt *descs, size_t n, uint8_t *arena, uint8_t *masks, int8_t *status,
                   uint32_t flags, void *stream) {
    if (!ctx || (n && (!descs || !arena))) return QPP_INTERNAL_ERROR;
    if ((flags & QPP_HP_MASK_OUT) && !masks) return QPP_INTERNAL_ERROR;
    if (n > UINT32_MAX) return QPP_INTERNAL_ERROR;
    if (!n) return QPP_OK;
    // FIPS mode refuses out-of-order nonces per packet (the packet stays plaintext): without a status array the call
    // could not say which, so it is refused (the reference fails such an encrypt call: aead/fips.rs)
    if (ctx->fips_live && !status && !(flags & QPP_ONLY_CHACHA)) return QPP_INTERNAL_ERROR;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    RC_TRY(flush_keys(ctx));
    StreamState *st = nullptr;
    RC_TRY(batch_stream(ctx, stream, &st));
    RC_TRY(enqueue_seal(ctx, st, descs, (uint32_t)n, arena, masks, status, flags));
    return note_work(ctx, st);
}

int qpp_open_batch(qpp_ctx *ctx, const qpp_pkt *descs, size_t n, uint8_t *arena, int8_t *status, uint32_t flags,
                   void *stream) {
    if (!ctx || (n && (!descs || !arena || !status))) return QPP_INTERNAL_ERROR;
    if (n > UINT32_MAX) return QPP_INTERNAL_ERROR;
    if (!n) return QPP_OK;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    RC_TRY(flush_keys(ctx));
    StreamState *st = nullptr;
    RC_TRY(batch_stream(ctx, stream, &st));
    RC_TRY(enqueue_open(ctx, st, descs, (uint32_t)n, arena, status, flags));
    return note_work(ctx, st);
}

int qpp_unprotect_open_batch(qpp_ctx *ctx, const qpp_rx_pkt *rx, size_t n, uint8_t *arena, qpp_pkt *descs_out,
                             int8_t *status, uint32_t flags, void *stream) {
    if (!ctx || (n && (!rx || !arena || !descs_out || !status))) return QPP_INTERNAL_ERROR;
    if (n > UINT32_MAX) return QPP_INTERNAL_ERROR;
    if (!n) return QPP_OK;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    RC_TRY(flush_keys(ctx));
    StreamState *st = nullptr;
    RC_TRY(batch_stream(ctx, stream, &st));
    // Any live AES packet key (any number of them, both sizes, beside ChaCha20 keys, any header-key suite) and a batch
    // of the quad kernel's size: ONE fused cooperative launch -- unprotect, group by the chosen key, open the AES
    // packets (quad.hip) -- and, when ChaCha20 packet keys are live, the ChaCha20 packets it sorted out opened by one
    // more launch on the same stream (no host round trip).  The same outputs as the launches below.  QPP_RX_FUSED=0
    // forces the multi-launch path (A/B, tests).
    const char *fz = getenv("QPP_RX_FUSED");
    const uint32_t a128 = ctx->live_by_suite[QPP_SUITE_TLS_AES_128_GCM_SHA256],
                   a256 = ctx->live_by_suite[QPP_SUITE_TLS_AES_256_GCM_SHA384];
    const bool chacha = !(flags & QPP_ONLY_AES) && ctx->live_by_suite[QPP_SUITE_TLS_CHACHA20_POLY1305_SHA256];
    if (!(flags & QPP_ONLY_CHACHA) && !(fz && fz[0] == '0') && a128 + a256 > 0 &&
        aes_path(ctx, (uint32_t)n) == AesPath::quad && ctx->key_cap <= quad_rx_max_keys()) {
        RC_TRY(ensure_plan(ctx, st, (uint32_t)n));  // perm
        const uint32_t kc = ctx->key_cap;
        if (st->rx_scratch_keys < kc) {
            HIP_TRY(ctx, hipStreamSynchronize(st->stream));  // the old scratch is no longer read
            dfree(ctx, st->rx_scratch);
            st->rx_scratch = nullptr;
            st->rx_scratch_keys = 0;
            HIP_TRY(ctx, dmalloc(ctx, &st->rx_scratch, 4 * (16 + 2 * (size_t)kc + 4 + 4 * ((size_t)kc + 1))));
            st->rx_scratch_keys = kc;
        }
        HIP_TRY(ctx, hipMemsetAsync(st->rx_scratch, 0, 4 * (16 + 2 * (size_t)kc), st->stream));
        {
            // The grid barriers need every workgroup resident: the grid is the CUs every resident server of the
            // device leaves, the device's previous fused receive is waited for (two at once would split the CUs), and
            // a server launched later waits for this one (srv_start) -- all under the device registry's lock
            DevServers &r = dev_servers(ctx->device);
            std::lock_guard<std::mutex> lk(r.mu);
            if (!r.rx_tail) HIP_TRY(ctx, hipEventCreateWithFlags(&r.rx_tail, hipEventDisableTiming));
            else HIP_TRY(ctx, hipStreamWaitEvent(st->stream, r.rx_tail, 0));
            const uint32_t busy = resident_wgs_locked(r), free_cu = ctx->n_cu > busy ? ctx->n_cu - busy : 1u;
            const uint32_t grid = std::min<uint32_t>(free_cu, std::max<uint32_t>(1, (uint32_t)((n + 191) / 192)));
            HIP_TRY(ctx, launch_aes_gcm_quad_rx(a256 ? (a128 ? 0u : 14u) : 10u, grid, st->stream, ctx->d_keys, kc, rx,
                                                (uint32_t)n, arena, descs_out, status, st->rx_scratch, st->plan.perm,
                                                ctx->d_diag, chacha, ctx->pow));
            HIP_TRY(ctx, hipEventRecord(r.rx_tail, st->stream));
        }
        if (chacha)
            HIP_TRY(ctx, launch_chacha_sel(ctx->d_keys, kc, descs_out, (uint32_t)n, arena, status, st->plan.perm,
                                           st->rx_scratch + 2, st->stream));
        return note_work(ctx, st);
    }
    // No AES record live at all (packet or header keys): every header and packet key a packet can name is ChaCha20,
    // so the ChaCha lane kernel unprotects and opens in ONE launch, whatever the key mix (per-lane keys, no plan).
    const bool no_aes = !ctx->live_by_suite[QPP_SUITE_TLS_AES_128_GCM_SHA256] &&
                        !ctx->live_by_suite[QPP_SUITE_TLS_AES_256_GCM_SHA384] &&
                        !ctx->hdr_live_by_suite[QPP_SUITE_TLS_AES_128_GCM_SHA256] &&
                        !ctx->hdr_live_by_suite[QPP_SUITE_TLS_AES_256_GCM_SHA384];
    if (no_aes && !(flags & QPP_ONLY_AES) && !(fz && fz[0] == '0') && n > (ctx->burst_max >> kChachaBurstShift)) {
        HIP_TRY(ctx, launch_chacha_rx(ctx->d_keys, ctx->key_cap, rx, (uint32_t)n, arena, descs_out, status, st->stream));
        return note_work(ctx, st);
    }
    // 1. header unprotection + PN expansion + key-phase choice -> descs_out (device); 2. the open kernels on them,
    // grouped by the chosen key like any batch (skipped packets keep their DECODE_ERROR status)
    HIP_TRY(ctx, launch_unprotect(ctx->d_keys, ctx->key_cap, rx, (uint32_t)n, arena, descs_out, status, st->stream));
    RC_TRY(enqueue_open(ctx, st, descs_out, (uint32_t)n, arena, status, flags));
    return note_work(ctx, st);
}

int qpp_pn_truncate(uint64_t pn, uint64_t largest_acked, uint64_t *truncated, size_t *pn_len) {
    // derive_truncation_range: (pn - largest) * 2 must fit the 1..4-byte encoding (mod.rs:81-93, packet_number_len.rs:163-172)
    if (!truncated || !pn_len) return QPP_INTERNAL_ERROR;
    pn &= kPnMask;
    largest_acked &= kPnMask;
    if (pn < largest_acked) return QPP_DECODE_ERROR;
    const uint64_t range = (pn - largest_acked) * 2;
    size_t len = 0;
    for (size_t b = 1; b <= 4 && !len; b++)
        if (range <= (1ull << (8 * b)) - 1) len = b;
    if (!len) return QPP_DECODE_ERROR;
    *pn_len = len;
    *truncated = pn & ((1ull << (8 * len)) - 1);
    return QPP_OK;
}

uint64_t qpp_pn_expand(uint64_t largest_acked, uint64_t truncated, size_t pn_len) {
    if (pn_len < 1 || pn_len > 4) return UINT64_MAX;
    return decode_packet_number(largest_acked & kPnMask, truncated, (uint32_t)(8 * pn_len));
}

int qpp_hp_mask_batch(qpp_ctx *ctx, const qpp_pkt *descs, size_t n, const uint8_t *arena, uint8_t *masks,
                      void *stream) {
    if (!ctx || (n && (!descs || !arena || !masks))) return QPP_INTERNAL_ERROR;
    if (!n) return QPP_OK;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    RC_TRY(flush_keys(ctx));
    StreamState *st = nullptr;
    RC_TRY(batch_stream(ctx, stream, &st));
    HIP_TRY(ctx, launch_hp_mask(ctx->d_keys, ctx->key_cap, descs, (uint32_t)n, arena, masks, st->stream));
    return note_work(ctx, st);
}

// ---------------------------------------------------------------- host pipeline (packets start and end in host memory)

int qpp_ctx_set_host_pipe(qpp_ctx *ctx, size_t chunk_packets, size_t chunk_bytes, size_t slots) {
    if (!ctx || !chunk_packets || chunk_packets > UINT32_MAX || chunk_bytes < 4096 || slots < 2 || slots > 16)
        return QPP_INTERNAL_ERROR;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    RC_TRY(servers_stop(ctx));
    RC_TRY(ctx_sync(ctx));
    if (!ctx->pipe) ctx->pipe = new HostPipe();
    pipe_release(ctx);
    ctx->pipe->chunk_packets = chunk_packets;
    ctx->pipe->chunk_bytes = chunk_bytes;
    ctx->pipe->nslots = slots;
    ctx->pipe->auto_chunk = false;
    return QPP_OK;
}

int qpp_host_batch_submit(qpp_ctx *ctx, const qpp_pkt *descs, size_t n, uint8_t *arena, uint8_t *masks,
                          int8_t *status, uint32_t flags, uint32_t ops, uint64_t *ticket) {
    if (!ctx || !ticket || (n && (!descs || !arena))) return QPP_INTERNAL_ERROR;
    if (!(ops & (QPP_OP_SEAL | QPP_OP_OPEN)) || (ops & ~(QPP_OP_SEAL | QPP_OP_OPEN))) return QPP_INTERNAL_ERROR;
    if ((flags & QPP_HP_MASK_OUT) && !(masks && (ops & QPP_OP_SEAL))) return QPP_INTERNAL_ERROR;
    if ((ops & QPP_OP_OPEN) && n && !status) return QPP_INTERNAL_ERROR;
    if ((ops & QPP_OP_SEAL) && n && !status && ctx->fips_live && !(flags & QPP_ONLY_CHACHA))
        return QPP_INTERNAL_ERROR;  // FIPS refusals are reported per packet (qpp_seal_batch)
    if ((ops & QPP_OP_SEAL) && (ops & QPP_OP_OPEN) && (flags & QPP_HP_APPLY)) return QPP_INTERNAL_ERROR;
    const bool by_conn = (flags & QPP_KEY_BY_CONN) != 0;
    if (by_conn && !ctx->connmap_n) return QPP_INTERNAL_ERROR;  // no connection table
    flags &= ~QPP_KEY_BY_CONN;
    *ticket = 0;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    if (!ctx->pipe) ctx->pipe = new HostPipe();
    HostPipe *p = ctx->pipe;
    RC_TRY(pipe_init(ctx));
    RC_TRY(flush_keys(ctx));
    StreamState *st = nullptr;
    RC_TRY(batch_stream(ctx, p->comp, &st));
    // chunks of consecutive packets: at most chunk_packets, span [lo, hi) of at most chunk_bytes; packets must be in
    // ascending, non-overlapping arena order so that spans of different chunks never overlap
    size_t cap = p->chunk_packets;
    if (p->auto_chunk) {
        const size_t keys = ctx->live_by_suite[QPP_SUITE_TLS_AES_128_GCM_SHA256] +
                            ctx->live_by_suite[QPP_SUITE_TLS_AES_256_GCM_SHA384];
        cap = std::min(p->chunk_packets, std::max<size_t>({(n + 15) / 16, 65536, 64 * keys}));
    }
    size_t i = 0;
    uint64_t prev_end = 0;
    while (i < n) {
        const size_t first = i;
        const uint64_t lo = descs[i].off;
        uint64_t hi = lo;
        while (i < n && i - first < cap) {
            const qpp_pkt &d = descs[i];
            const uint64_t end = (uint64_t)d.off + d.aad_len + d.pt_len + 16;
            if (d.off < prev_end) return QPP_INTERNAL_ERROR;  // out of order or overlapping
            if (end - lo > p->chunk_bytes) {
                if (i == first) return QPP_INTERNAL_ERROR;  // one packet larger than a chunk buffer
                break;
            }
            hi = std::max(hi, end);
            prev_end = end;
            i++;
        }
        const uint32_t cn = (uint32_t)(i - first);
        PipeSlot &sl = p->slots[p->next];
        p->next = (p->next + 1) % p->slots.size();
        // the slot's previous chunk must be back in host memory before its buffers are overwritten (device-side wait)
        if (sl.busy) HIP_TRY(ctx, hipStreamWaitEvent(p->h2d, sl.d2h, 0));
        HIP_TRY(ctx, hipMemcpyAsync(sl.arena, arena + lo, hi - lo, hipMemcpyHostToDevice, p->h2d));
        HIP_TRY(ctx, hipMemcpyAsync(sl.descs, descs + first, sizeof(qpp_pkt) * cn, hipMemcpyHostToDevice, p->h2d));
        HIP_TRY(ctx, hipEventRecord(sl.h2d, p->h2d));
        HIP_TRY(ctx, hipStreamWaitEvent(p->comp, sl.h2d, 0));
        if (by_conn)
            HIP_TRY(ctx, launch_conn_remap(sl.descs, cn, ctx->d_connmap, (uint32_t)ctx->connmap_n, p->comp));
        uint8_t *base = sl.arena - lo;  // descriptor offsets stay absolute: the kernels address base + off
        if (ops & QPP_OP_SEAL)
            RC_TRY(enqueue_seal(ctx, st, sl.descs, cn, base, sl.masks, (ops & QPP_OP_OPEN) ? nullptr : sl.status,
                                flags));
        if (ops & QPP_OP_OPEN)
            RC_TRY(enqueue_open(ctx, st, sl.descs, cn, base, sl.status, flags & ~(QPP_HP_MASK_OUT | QPP_HP_APPLY)));
        HIP_TRY(ctx, hipEventRecord(sl.comp, p->comp));
        HIP_TRY(ctx, hipStreamWaitEvent(p->d2h, sl.comp, 0));
        HIP_TRY(ctx, hipMemcpyAsync(arena + lo, sl.arena, hi - lo, hipMemcpyDeviceToHost, p->d2h));
        if ((flags & QPP_HP_MASK_OUT) && masks)
            HIP_TRY(ctx, hipMemcpyAsync(masks + 5 * first, sl.masks, 5 * (size_t)cn, hipMemcpyDeviceToHost, p->d2h));
        if (status) HIP_TRY(ctx, hipMemcpyAsync(status + first, sl.status, cn, hipMemcpyDeviceToHost, p->d2h));
        HIP_TRY(ctx, hipEventRecord(sl.d2h, p->d2h));
        sl.busy = true;
    }
    RC_TRY(note_work(ctx, st));
    hipEvent_t done = get_event(ctx);
    if (!done) return QPP_DEVICE_ERROR;
    HIP_TRY(ctx, hipEventRecord(done, p->d2h));
    *ticket = p->next_ticket++;
    p->tickets[*ticket] = done;
    return QPP_OK;
}

int qpp_ctx_set_conn_keys(qpp_ctx *ctx, const uint32_t *slots, size_t n) {
    if (!ctx || !n || !slots || n > UINT32_MAX) return QPP_INTERNAL_ERROR;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    if (!ctx->pipe) ctx->pipe = new HostPipe();
    RC_TRY(pipe_init(ctx));
    hipStream_t s = ctx->pipe->comp;  // the remap launches' stream: earlier batches read the old table first
    if (n > ctx->connmap_cap) {
        HIP_TRY(ctx, hipStreamSynchronize(s));
        dfree(ctx, ctx->d_connmap);  // (behind every stream: conn-keyed batches of any stream read it)
        ctx->d_connmap = nullptr;
        ctx->connmap_cap = ctx->connmap_n = 0;
        const size_t cap = std::max<size_t>(n, 1024);
        HIP_TRY(ctx, dmalloc(ctx, &ctx->d_connmap, 4 * cap));
        ctx->connmap_cap = cap;
    }
    // through the pinned stage: the caller may reuse `slots` on return (the previous copy from the stage is waited
    // for first -- a host wait only when two tables are swapped back to back)
    if (!ctx->connstage_ev) HIP_TRY(ctx, hipEventCreateWithFlags(&ctx->connstage_ev, hipEventDisableTiming));
    if (ctx->connstage_used) HIP_TRY(ctx, hipEventSynchronize(ctx->connstage_ev));
    ctx->connstage_used = false;
    if (n > ctx->connstage_cap) {
        hfree(ctx, ctx->h_connstage);
        ctx->h_connstage = nullptr;
        ctx->connstage_cap = 0;
        const size_t cap = std::max<size_t>(n, 1024);
        HIP_TRY(ctx, hmalloc(&ctx->h_connstage, 4 * cap, hipHostMallocDefault));
        ctx->connstage_cap = cap;
    }
    memcpy(ctx->h_connstage, slots, 4 * n);
    HIP_TRY(ctx, hipMemcpyAsync(ctx->d_connmap, ctx->h_connstage, 4 * n, hipMemcpyHostToDevice, s));
    HIP_TRY(ctx, hipEventRecord(ctx->connstage_ev, s));
    ctx->connstage_used = true;
    ctx->connmap_n = n;
    return QPP_OK;
}

int qpp_host_batch_query(qpp_ctx *ctx, uint64_t ticket, int *done) {
    if (!ctx || !done || !ctx->pipe) return QPP_INTERNAL_ERROR;
    auto it = ctx->pipe->tickets.find(ticket);
    if (it == ctx->pipe->tickets.end()) return QPP_INTERNAL_ERROR;
    const hipError_t q = hipEventQuery(it->second);
    if (q == hipErrorNotReady) { *done = 0; return QPP_OK; }
    HIP_TRY(ctx, q);
    *done = 1;
    return QPP_OK;
}

int qpp_host_batch_wait(qpp_ctx *ctx, uint64_t ticket) {
    if (!ctx || !ctx->pipe) return QPP_INTERNAL_ERROR;
    auto it = ctx->pipe->tickets.find(ticket);
    if (it == ctx->pipe->tickets.end()) return QPP_INTERNAL_ERROR;
    hipEvent_t e = it->second;
    ctx->pipe->tickets.erase(it);
    const hipError_t r = hipEventSynchronize(e);
    put_event(ctx, e);
    HIP_TRY(ctx, r);
    return QPP_OK;
}

// ---------------------------------------------------------------- plumbing

int qpp_dev_alloc(qpp_ctx *ctx, size_t bytes, void **out) {
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    HIP_TRY(ctx, dmalloc(ctx, out, bytes));
    return QPP_OK;
}
void qpp_dev_free(qpp_ctx *ctx, void *ptr) {
    if (!ptr) return;
    hipSetDevice(ctx->device);
    dfree(ctx, ptr);  // behind the work every stream of the context has been given so far
}
int qpp_host_alloc(qpp_ctx *ctx, size_t bytes, void **out) {
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    HIP_TRY(ctx, hmalloc(out, bytes ? bytes : 1, hipHostMallocDefault));
    return QPP_OK;
}
void qpp_host_free(qpp_ctx *ctx, void *ptr) {
    if (!ptr) return;
    if (!ctx) {
        hipHostFree(ptr);
        return;
    }
    hfree(ctx, ptr);  // (parked while a server of the device is resident)
}
int qpp_memcpy_d2d(qpp_ctx *ctx, void *dst, const void *src, size_t bytes, void *stream) {
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    HIP_TRY(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToDevice, user_stream(ctx, stream)));
    return QPP_OK;
}

int qpp_memcpy_h2d(qpp_ctx *ctx, void *dst, const void *src, size_t bytes, void *stream) {
    HIP_TRY(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, user_stream(ctx, stream)));
    return QPP_OK;
}
int qpp_memcpy_d2h(qpp_ctx *ctx, void *dst, const void *src, size_t bytes, void *stream) {
    HIP_TRY(ctx, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, user_stream(ctx, stream)));
    return QPP_OK;
}
int qpp_memset_d(qpp_ctx *ctx, void *dst, int value, size_t bytes, void *stream) {
    HIP_TRY(ctx, hipMemsetAsync(dst, value, bytes, user_stream(ctx, stream)));
    return QPP_OK;
}
int qpp_stream_create(qpp_ctx *ctx, void **out) {
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    hipStream_t s;
    HIP_TRY(ctx, hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    user_stream(ctx, (void *)s);
    *out = (void *)s;
    return QPP_OK;
}
void qpp_stream_destroy(qpp_ctx *ctx, void *stream) {
    if (!stream) return;
    hipStream_t s = (hipStream_t)stream;
    if (ctx && s != ctx->stream) {
        hipStreamSynchronize(s);  // its batches are done: its plan scratch and last-batch event can go
        for (size_t i = 0; i < ctx->streams.size(); i++) {
            StreamState *st = ctx->streams[i];
            if (st->stream != s) continue;
            free_stream_state(ctx, st);
            ctx->streams.erase(ctx->streams.begin() + (long)i);
            break;
        }
        ctx->user_streams.erase(std::remove(ctx->user_streams.begin(), ctx->user_streams.end(), s),
                                ctx->user_streams.end());
    }
    hipStreamDestroy(s);
}
int qpp_stream_synchronize(qpp_ctx *ctx, void *stream) {
    HIP_TRY(ctx, hipStreamSynchronize(stream ? (hipStream_t)stream : ctx->stream));
    return QPP_OK;
}
int qpp_event_create(qpp_ctx *ctx, void **out) {
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    hipEvent_t e;
    HIP_TRY(ctx, hipEventCreate(&e));
    *out = (void *)e;
    return QPP_OK;
}
void qpp_event_destroy(qpp_ctx *, void *event) {
    if (event) hipEventDestroy((hipEvent_t)event);
}
int qpp_event_record(qpp_ctx *ctx, void *event, void *stream) {
    HIP_TRY(ctx, hipEventRecord((hipEvent_t)event, user_stream(ctx, stream)));
    return QPP_OK;
}
int qpp_event_elapsed_ms(qpp_ctx *ctx, void *start, void *stop, float *ms) {
    HIP_TRY(ctx, hipEventSynchronize((hipEvent_t)stop));
    HIP_TRY(ctx, hipEventElapsedTime(ms, (hipEvent_t)start, (hipEvent_t)stop));
    return QPP_OK;
}

int qpp_stream_wait_event(qpp_ctx *ctx, void *stream, void *event) {
    HIP_TRY(ctx, hipStreamWaitEvent(user_stream(ctx, stream), (hipEvent_t)event, 0));
    return QPP_OK;
}

}  // extern "C"

// ---------------------------------------------------------------- deferred transmit queue

// One in-flight flush of a txq: its descriptors and (zero-copy) plan in pinned memory, the device copies for the DMA
// path, the stream it went out on and the event that ends it.
struct TxqSlot {
    qpp_pkt *h_desc = nullptr, *d_desc = nullptr, *v_desc = nullptr;
    uint32_t *h_perm = nullptr;  // pinned: perm[max_packets] | n_work | WorkItem work[max_packets + 1]
    WorkItem *h_work = nullptr;
    uint32_t *h_nwork = nullptr;
    PlanBuffers v_plan{};
    hipStream_t stream = nullptr;
    hipEvent_t done = nullptr;
    uint64_t first = 0, last = 0;  // tickets (bursts) of the flush that last used this slot (0: never)
    uint32_t *h_refused = nullptr;  // pinned: packets of the flush the FIPS nonce-order gate refused
    bool busy = false;    // `done` recorded and not yet seen complete
};

struct qpp_txq {
    qpp_ctx *ctx = nullptr;
    size_t ring_bytes = 0, max_packets = 0;
    uint8_t *h_ring = nullptr, *d_ring = nullptr, *v_ring = nullptr;
    // flushes in flight: the batch being pushed fills slots[cur]; flush_async sends it and moves to the next slot
    std::vector<TxqSlot> slots;
    std::vector<hipStream_t> streams;
    size_t cur = 0;
    uint64_t next_ticket = 1;
    // bursts flushed into slots[cur] but not yet submitted (coalescing): tickets [pend_first, pend_last]
    uint64_t pend_first = 0, pend_last = 0;
    uint32_t pend_bursts = 0, coalesce = 1;
    size_t count = 0, lo = SIZE_MAX, hi = 0;
    size_t count_at_ticket = 0;  // q->count at the last flush_async (packets pushed since belong to the next ticket)
    uint32_t suites = 0;
    // zero-copy flush of small bursts: the kernels read and write the pinned ring, descriptors and a host-built
    // plan directly over PCIe (no DMA copies, no plan launches)
    uint32_t zc_max = 0;
    std::vector<uint32_t> order;
    std::vector<std::pair<size_t, size_t>> runs;  // DMA path: the flush's contiguous packet byte ranges
    // Persistent server (qpp_txq_create_persistent; burst.hip txq_server_kernel): flushes of AES packets are posted
    // through per-workgroup slots in pinned memory instead of launched.  One posted flush at a time: its plan (work items and
    // key-sorted descriptors, pinned) is rewritten only once `done` shows the previous one sealed.
    bool persistent = false;
    TxsMail *h_mail = nullptr, *v_mail = nullptr;
    TxsSlot *h_slots = nullptr, *v_slots = nullptr;  // one per server workgroup
    WorkItem *h_items = nullptr, *v_items = nullptr;
    qpp_pkt *h_sdesc = nullptr, *v_sdesc = nullptr;
    hipStream_t srv_stream = nullptr;
    bool srv_running = false;           // launched and not yet seen to have ended
    std::atomic<bool> srv_launched{false};  // the same, readable by other contexts' threads (device registry)
    std::atomic<bool> evicted{false};       // release() made the server leave (another thread): srv_running is stale
    const DevKey *srv_keys = nullptr;   // the key table the running server reads
    uint32_t srv_seq = 0;               // seq of the last flush or stop written into the slots
    uint32_t srv_posted = 0;            // seq of the last flush posted (0: none)
    uint64_t srv_first = 0, srv_last = 0;  // its tickets
    uint32_t srv_epoch = 0;             // key epoch posted with the flushes (8 bits)
    uint64_t srv_key_gen = ~0ull;       // ctx->key_gen the server's epoch stands for
    uint32_t srv_wgs = 16, srv_idle_ticks = 0;
    std::chrono::steady_clock::time_point srv_last_post{};  // the server may leave idle_ticks after it
    std::chrono::microseconds srv_host_idle{0};             // a quarter of that: past it, restart before posting
    uint64_t n_server = 0, n_launch = 0, n_starts = 0;  // flushes posted / launched; server launches
    uint64_t n_oneshots = 0;            // of which one-shot launches finishing a posted flush (srv_oneshot)
    hipEvent_t oneshot_ev = nullptr;    // behind the latest one
};

namespace {

const std::vector<hipStream_t> &txq_streams(const qpp_txq *q) { return q->streams; }

constexpr int kNoServerSlot = 1000;  // (internal) srv_start: every server slot of the device is taken

// launched and its stream still busy: read-only on the queue, safe for another context's thread (registry lock held)
bool srv_resident(const qpp_txq *q) {
    return q->srv_launched.load(std::memory_order_acquire) && hipStreamQuery(q->srv_stream) == hipErrorNotReady;
}
uint32_t resident_wgs_locked(const DevServers &r) {
    uint32_t w = 0;
    for (const qpp_txq *o : r.queues)
        if (srv_resident(o)) w += o->srv_wgs;
    return w;
}

// Frees p at once when no server of the device is resident, else parks it, up to parked_max() bytes per device.  Past
// that bound the device's resident servers -- every context's -- are EVICTED: the eviction word makes each leave at its
// next poll that finds no complete flush (a flush it has seen is finished first), their streams are waited for (a
// poll, or the flush in hand: microseconds), and only then does hipFree run -- it never waits for a server that keeps
// being fed.  An evicted queue's owner relaunches its server at its next post (srv_prepare),
// and a flush posted while its server left is picked up by the relaunched one (srv_wait).  p = nullptr only frees what
// is parked, if it can.  Under the registry lock throughout, so no server starts between the wait and the free.
void release(qpp_ctx *ctx, void *p, bool pinned) {
    DevServers &r = dev_servers(ctx->device);
    std::unique_lock<std::mutex> lk(r.mu);
    auto resident = [&r] {
        for (const qpp_txq *o : r.queues)
            if (srv_resident(o)) return true;
        return false;
    };
    size_t bytes = p ? take_size(p) : 0;
    if (p && !bytes) bytes = size_t(1) << 20;  // (not allocated through this library: counted as 1 MiB)
    if (resident()) {
        if (!p) return;
        if (r.parked_bytes + bytes <= parked_max()) {
            r.parked.emplace_back(p, pinned);
            r.parked_bytes += bytes;
            return;
        }
        if (r.h_evict) {
            __atomic_store_n(r.h_evict, 1u, __ATOMIC_RELEASE);
            for (qpp_txq *o : r.queues) {
                if (!o->srv_launched.load(std::memory_order_acquire)) continue;
                hipStreamSynchronize(o->srv_stream);  // (its server leaves at its next poll)
                o->evicted.store(true, std::memory_order_release);
            }
            __atomic_store_n(r.h_evict, 0u, __ATOMIC_RELEASE);
            r.evictions++;
        }
    }
    for (const auto &x : r.parked) {
        if (x.second) hipHostFree(x.first);
        else hipFree(x.first);
    }
    r.parked.clear();
    r.parked_bytes = 0;
    if (p) {
        if (pinned) hipHostFree(p);
        else hipFree(p);
    }
}

uint32_t srv_next(uint32_t s) { return s + 1u ? s + 1u : 1u; }  // 0 is never a flush's seq

bool srv_alive(qpp_txq *q) {
    if (!q->srv_running) return false;
    if (hipStreamQuery(q->srv_stream) == hipErrorNotReady) return true;
    q->srv_running = false;  // it ended on its own (idle timeout), or failed (the next launch reports that)
    q->srv_launched.store(false, std::memory_order_release);
    return false;
}

// Launches the server unless it runs.  A flush posted but not done (posted while the last server was leaving on its
// idle timeout) is picked up by the new one: it starts with seq0 != the posted seq.
// every workgroup has sealed the flush with this seq
bool srv_done(const qpp_txq *q, uint32_t seq) {
    for (uint32_t b = 0; b < q->srv_wgs; b++)
        if (__atomic_load_n(&q->h_slots[b].done, __ATOMIC_ACQUIRE) != seq) return false;
    return true;
}

// force: a posted flush waits for this server (srv_wait's restart), so it starts even past the device's server slots
int srv_start(qpp_txq *q, bool force = false) {
    // (no stream query while the server is believed running: a server that left on its idle timeout is found by
    // srv_wait's slow path, which relaunches it behind the posted flush)
    if (q->srv_running && q->evicted.exchange(false, std::memory_order_acq_rel)) srv_alive(q);  // (it left)
    if (q->srv_running) return QPP_OK;
    qpp_ctx *ctx = q->ctx;
    DevServers &r = dev_servers(ctx->device);
    std::lock_guard<std::mutex> lk(r.mu);
    if (!force) {
        uint32_t n = 0;
        for (const qpp_txq *o : r.queues)
            if (o != q && srv_resident(o)) n++;
        if (n >= server_slots()) return kNoServerSlot;
    }
    // behind the device's latest fused receive (its grid did not count this server's CUs)
    if (r.rx_tail) HIP_TRY(ctx, hipStreamWaitEvent(q->srv_stream, r.rx_tail, 0));
    const bool pending = q->srv_posted && !srv_done(q, q->srv_posted);
    const uint32_t seq0 = pending ? q->srv_posted - 1u : q->srv_seq;
    HIP_TRY(ctx, launch_txq_server(ctx->d_keys, ctx->pow, q->v_mail, q->v_slots, q->v_items, q->v_sdesc, q->v_ring,
                                   (uint32_t)std::min<size_t>(q->ring_bytes, UINT32_MAX), seq0, q->srv_idle_ticks,
                                   q->srv_wgs, r.v_evict, q->srv_stream));
    q->srv_running = true;
    q->srv_launched.store(true, std::memory_order_release);
    q->srv_keys = ctx->d_keys;
    q->srv_last_post = std::chrono::steady_clock::now();  // (its idle clock starts now)
    q->n_starts++;
    return QPP_OK;
}

// A posted flush whose server left before every workgroup saw it (idle exit, or evicted by release) while every
// server slot of the device is taken: a relaunched server could land on a hardware queue a fed server holds and wait
// for that server's exit.  So the flush is finished by a ONE-SHOT launch of the server kernel (idle 0: it
// serves the posted flush in the workgroups whose `done` does not show it yet, then leaves) on the context's own
// normal-priority stream.  At most one in flight per queue.
int srv_oneshot(qpp_txq *q) {
    qpp_ctx *ctx = q->ctx;
    if (q->oneshot_ev && hipEventQuery(q->oneshot_ev) == hipErrorNotReady) return QPP_OK;
    if (!q->oneshot_ev) HIP_TRY(ctx, hipEventCreateWithFlags(&q->oneshot_ev, hipEventDisableTiming));
    DevServers &r = dev_servers(ctx->device);
    std::lock_guard<std::mutex> lk(r.mu);
    if (r.rx_tail) HIP_TRY(ctx, hipStreamWaitEvent(ctx->stream, r.rx_tail, 0));
    HIP_TRY(ctx, launch_txq_server(ctx->d_keys, ctx->pow, q->v_mail, q->v_slots, q->v_items, q->v_sdesc, q->v_ring,
                                   (uint32_t)std::min<size_t>(q->ring_bytes, UINT32_MAX), q->srv_posted - 1u, 0u,
                                   q->srv_wgs, r.v_evict, ctx->stream));
    HIP_TRY(ctx, hipEventRecord(q->oneshot_ev, ctx->stream));
    q->n_starts++;
    q->n_oneshots++;
    r.oneshots++;
    return QPP_OK;
}

// Host wait for the flush with this seq (spinning on the pinned `done` word: no interrupt, no runtime call).
int srv_wait(qpp_txq *q, uint32_t seq) {
    if (!seq) return QPP_OK;
    std::chrono::steady_clock::time_point t0{};
    for (uint64_t spin = 0;; spin++) {
        if (srv_done(q, seq)) return QPP_OK;
        if ((spin & 4095u) == 4095u) {
            // it left (idle, evicted) before this flush was seen: a new one takes it -- unless a one-shot launch is
            // still on it (two kernels must never serve one flush: the ring is sealed in place)
            const bool oneshot = q->oneshot_ev && hipEventQuery(q->oneshot_ev) == hipErrorNotReady;
            if (!oneshot && !srv_alive(q)) {
                int rc = srv_start(q);
                if (rc == kNoServerSlot) rc = srv_oneshot(q);
                RC_TRY(rc);
            }
            const auto now = std::chrono::steady_clock::now();
            if (spin == 4095u) t0 = now;
            else if (now - t0 > std::chrono::seconds(10)) {
                q->ctx->last_error = "txq server: flush not completed within 10 s";
                return QPP_DEVICE_ERROR;
            }
        }
        __builtin_ia32_pause();
    }
}

int srv_stop(qpp_txq *q) {
    if (!q->srv_running) return QPP_OK;
    RC_TRY(srv_wait(q, q->srv_posted));
    if (!srv_alive(q)) return QPP_OK;
    q->srv_seq = srv_next(q->srv_seq);
    for (uint32_t b = 0; b < q->srv_wgs; b++) {
        q->h_slots[b].word = kTxsStop;
        __atomic_store_n(&q->h_slots[b].seq, q->srv_seq, __ATOMIC_RELEASE);
    }
    HIP_TRY(q->ctx, hipStreamSynchronize(q->srv_stream));
    q->srv_running = false;
    q->srv_launched.store(false, std::memory_order_release);
    return QPP_OK;
}

int servers_stop(qpp_ctx *ctx) {
    for (qpp_txq *q : ctx->servers) RC_TRY(srv_stop(q));
    return QPP_OK;
}
int servers_quiesce(qpp_ctx *ctx) {
    for (qpp_txq *q : ctx->servers) RC_TRY(srv_wait(q, q->srv_posted));
    return QPP_OK;
}
uint32_t servers_cu(const qpp_ctx *ctx) {  // every resident server of the device, any context
    DevServers &r = dev_servers(ctx->device);
    std::lock_guard<std::mutex> lk(r.mu);
    return resident_wgs_locked(r);
}

}  // namespace

extern "C" {

int qpp_txq_create(qpp_ctx *ctx, size_t ring_bytes, size_t max_packets, qpp_txq **out) {
    return qpp_txq_create_async(ctx, ring_bytes, max_packets, 1, out);
}

}  // extern "C"

// ring_flags: hipHostMallocDefault (launched flushes), or coherent + mapped (a server's ring, see txq_make_server)
static int txq_create(qpp_ctx *ctx, size_t ring_bytes, size_t max_packets, size_t in_flight, unsigned ring_flags,
                      qpp_txq **out) {
    if (!ctx || !out || !ring_bytes || !max_packets || ring_bytes > UINT32_MAX || max_packets > UINT32_MAX ||
        !in_flight || in_flight > 64)
        return QPP_INTERNAL_ERROR;
    *out = nullptr;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    qpp_txq *q = new qpp_txq();
    q->ctx = ctx;
    q->ring_bytes = ring_bytes;
    q->max_packets = max_packets;
    void *v = nullptr;
    auto bad = [&](hipError_t e, const char *what) {
        if (!fail(ctx, e, what)) return false;
        qpp_txq_destroy(q);
        return true;
    };
    if (bad(hmalloc(&q->h_ring, ring_bytes, ring_flags), "txq ring") ||
        bad(dmalloc(ctx, &q->d_ring, ring_bytes), "txq ring") || bad(hipHostGetDevicePointer(&v, q->h_ring, 0), "ring view"))
        return QPP_DEVICE_ERROR;
    q->v_ring = (uint8_t *)v;
    // one stream per in-flight flush up to 4 (the hardware queues a process gets), shared round-robin beyond
    const size_t nstreams = in_flight < 4 ? in_flight : 4;
    for (size_t i = 0; i < nstreams; i++) {
        hipStream_t st = nullptr;
        if (bad(hipStreamCreateWithFlags(&st, hipStreamNonBlocking), "txq stream")) return QPP_DEVICE_ERROR;
        q->streams.push_back(st);
    }
    q->slots.resize(in_flight);
    for (size_t i = 0; i < in_flight; i++) {
        TxqSlot &sl = q->slots[i];
        sl.stream = q->streams[i % nstreams];
        if (bad(hmalloc(&sl.h_desc, sizeof(qpp_pkt) * max_packets, hipHostMallocDefault), "txq descs") ||
            bad(dmalloc(ctx, &sl.d_desc, sizeof(qpp_pkt) * max_packets), "txq descs") ||
            bad(hmalloc(&sl.h_perm, 4 * (max_packets + 4) + sizeof(WorkItem) * (max_packets + 1),
                              hipHostMallocDefault), "txq plan") ||
            bad(hipEventCreateWithFlags(&sl.done, hipEventDisableTiming), "txq event") ||
            bad(hmalloc(&sl.h_refused, 64, hipHostMallocDefault), "txq refused count"))
            return QPP_DEVICE_ERROR;
        *sl.h_refused = 0;
        sl.h_nwork = sl.h_perm + max_packets;
        sl.h_work = (WorkItem *)(sl.h_perm + max_packets + 4);  // 16-byte aligned
        if (bad(hipHostGetDevicePointer(&v, sl.h_desc, 0), "txq desc view")) return QPP_DEVICE_ERROR;
        sl.v_desc = (qpp_pkt *)v;
        if (bad(hipHostGetDevicePointer(&v, sl.h_perm, 0), "txq plan view")) return QPP_DEVICE_ERROR;
        sl.v_plan.perm = (uint32_t *)v;
        sl.v_plan.n_work = sl.v_plan.perm + max_packets;
        sl.v_plan.work = (WorkItem *)(sl.v_plan.perm + max_packets + 4);
    }
    q->zc_max = kTxqZeroCopyMax;
    if (const char *e = getenv("QPP_TXQ_ZC_MAX")) q->zc_max = (uint32_t)strtoul(e, nullptr, 10);
    q->order.reserve(max_packets);
    memset(q->h_ring, 0, ring_bytes);
    ctx->txqs.push_back(q);
    *out = q;
    return QPP_OK;
}

extern "C" {

int qpp_txq_create_async(qpp_ctx *ctx, size_t ring_bytes, size_t max_packets, size_t in_flight, qpp_txq **out) {
    return txq_create(ctx, ring_bytes, max_packets, in_flight, hipHostMallocDefault, out);
}

void qpp_txq_destroy(qpp_txq *q) {
    if (!q) return;
    hipSetDevice(q->ctx->device);
    {
        std::vector<qpp_txq *> &all = q->ctx->txqs;
        all.erase(std::remove(all.begin(), all.end(), q), all.end());
    }
    quiet_for_free(q->ctx);  // this queue's server (and the context's others: restarted by their next call)
    if (q->persistent) {
        srv_stop(q);
        std::vector<qpp_txq *> &v = q->ctx->servers;
        v.erase(std::remove(v.begin(), v.end(), q), v.end());
        {
            DevServers &r = dev_servers(q->ctx->device);
            std::lock_guard<std::mutex> lk(r.mu);
            r.queues.erase(std::remove(r.queues.begin(), r.queues.end(), q), r.queues.end());
        }
        if (q->srv_stream) { hipStreamSynchronize(q->srv_stream); hipStreamDestroy(q->srv_stream); }
        if (q->oneshot_ev) { hipEventSynchronize(q->oneshot_ev); hipEventDestroy(q->oneshot_ev); }
        hfree(q->ctx, q->h_mail);
        if (q->h_slots) { secure_zero(q->h_slots, sizeof(TxsSlot) * q->srv_wgs); hfree(q->ctx, q->h_slots); }
        hfree(q->ctx, q->h_items);
        if (q->h_sdesc) { secure_zero(q->h_sdesc, sizeof(qpp_pkt) * q->max_packets * kTxsWaves); hfree(q->ctx, q->h_sdesc); }
    }
    for (hipStream_t st : q->streams) hipStreamSynchronize(st);
    if (q->h_ring) { secure_zero(q->h_ring, q->ring_bytes); hfree(q->ctx, q->h_ring); }
    if (q->d_ring) {
        hipMemsetAsync(q->d_ring, 0, q->ring_bytes, q->ctx->stream);
        hipStreamSynchronize(q->ctx->stream);
        dfree(q->ctx, q->d_ring);
    }
    for (TxqSlot &sl : q->slots) {
        hfree(q->ctx, sl.h_desc);
        dfree(q->ctx, sl.d_desc);  // (the queue's streams are synchronized above)
        hfree(q->ctx, sl.h_perm);
        if (sl.done) hipEventDestroy(sl.done);
        hfree(q->ctx, sl.h_refused);
    }
    for (hipStream_t st : q->streams) {
        // the stream's StreamState (plan scratch of the DMA path) goes with it
        qpp_stream_destroy(q->ctx, (void *)st);
    }
    delete q;
}

uint8_t *qpp_txq_ring(qpp_txq *q) { return q ? q->h_ring : nullptr; }
size_t qpp_txq_pending(const qpp_txq *q) { return q ? q->count - q->count_at_ticket : 0; }

int qpp_txq_push(qpp_txq *q, const qpp_key *key, uint64_t pn, size_t off, size_t header_len, size_t pn_len,
                 size_t payload_len) {
    if (!q || !key || key->ctx != q->ctx) return QPP_INTERNAL_ERROR;
    if (q->count >= q->max_packets) return QPP_INTERNAL_ERROR;  // flush first
    if (pn_len < 1 || pn_len > 4 || header_len + pn_len > 0xffff || payload_len > 0xffff) return QPP_INTERNAL_ERROR;
    const size_t end = off + header_len + pn_len + payload_len + 16;
    if (end > q->ring_bytes || end < off) return QPP_INTERNAL_ERROR;
    if (payload_len + pn_len < 4) return QPP_DECODE_ERROR;  // the sample at header_len + 4 must fit
    qpp_pkt &d = q->slots[q->cur].h_desc[q->count++];
    d = qpp_pkt{};
    d.pn = pn;
    d.key_idx = key->slot;
    d.off = (uint32_t)off;
    d.aad_len = (uint16_t)(header_len + pn_len);
    d.pt_len = (uint16_t)payload_len;
    d.pn_len = (uint8_t)pn_len;
    q->lo = std::min(q->lo, off);
    q->hi = std::max(q->hi, end);
    q->suites |= 1u << key->suite;
    return QPP_OK;
}

int qpp_txq_push_scatter(qpp_txq *q, const qpp_key *key, uint64_t pn, size_t off, size_t header_len, size_t pn_len,
                         size_t inline_len, const uint8_t *extra, size_t extra_len) {
    if (!q || (extra_len && !extra)) return QPP_INTERNAL_ERROR;
    const size_t payload_len = inline_len + extra_len;
    if (payload_len < inline_len || off > q->ring_bytes || header_len + pn_len > q->ring_bytes - off ||
        inline_len > q->ring_bytes - off - header_len - pn_len)
        return QPP_INTERNAL_ERROR;
    const size_t at = off + header_len + pn_len + inline_len;
    RC_TRY(qpp_txq_push(q, key, pn, off, header_len, pn_len, payload_len));  // every range / capacity check
    if (extra_len) memcpy(q->h_ring + at, extra, extra_len);  // the ring holds it through end + 16 (checked above)
    return QPP_OK;
}

int qpp_txq_push_descs(qpp_txq *q, const qpp_pkt *descs, size_t n) {
    if (!q || (n && !descs)) return QPP_INTERNAL_ERROR;
    if (n > q->max_packets - q->count) return QPP_INTERNAL_ERROR;  // flush first
    qpp_ctx *ctx = q->ctx;
    for (size_t i = 0; i < n; i++) {  // the checks of qpp_txq_push, all before anything is queued
        const qpp_pkt &d = descs[i];
        if (d.key_idx >= ctx->key_cap || ctx->h_keys[d.key_idx].live != 1) return QPP_INTERNAL_ERROR;
        if (d.pn_len < 1 || d.pn_len > 4 || d.aad_len < d.pn_len || d.flags) return QPP_INTERNAL_ERROR;
        const size_t end = (size_t)d.off + d.aad_len + d.pt_len + 16;
        if (end > q->ring_bytes) return QPP_INTERNAL_ERROR;
        if ((size_t)d.pt_len + d.pn_len < 4) return QPP_DECODE_ERROR;
    }
    memcpy(q->slots[q->cur].h_desc + q->count, descs, sizeof(qpp_pkt) * n);
    for (size_t i = 0; i < n; i++) {
        const qpp_pkt &d = descs[i];
        q->lo = std::min<size_t>(q->lo, d.off);
        q->hi = std::max<size_t>(q->hi, (size_t)d.off + d.aad_len + d.pt_len + 16);
        q->suites |= 1u << ctx->h_keys[d.key_idx].suite;
    }
    q->count += n;
    return QPP_OK;
}

// Zero-copy flush: host plan (AES packets grouped by key, work items of whole waves) in the slot's pinned memory,
// then the burst kernel (AES) and the ChaCha kernel on the pinned ring itself; one launch per suite family.
static int txq_enqueue_zero_copy(qpp_txq *q, TxqSlot &sl, StreamState *st, uint32_t n) {
    qpp_ctx *ctx = q->ctx;
    hipStream_t s = sl.stream;
    const qpp_pkt *descs = sl.v_desc;
    RC_TRY(fips_gate(ctx, st, descs, n, nullptr, st->fips_refused));
    if (q->suites & kAesSuites) {
        std::vector<uint32_t> &ord = q->order;
        ord.clear();
        for (uint32_t i = 0; i < n; i++)
            if (is_aes(ctx->h_keys[sl.h_desc[i].key_idx].suite)) ord.push_back(i);
        std::stable_sort(ord.begin(), ord.end(),
                         [&sl](uint32_t a, uint32_t b) { return sl.h_desc[a].key_idx < sl.h_desc[b].key_idx; });
        const uint32_t per = burst_packets_per_item((uint32_t)ord.size(), ctx->n_cu);
        uint32_t items = 0, keys = 0;
        for (uint32_t i = 0; i < ord.size();) {
            const uint32_t slot = sl.h_desc[ord[i]].key_idx;
            uint32_t j = i;
            while (j < ord.size() && sl.h_desc[ord[j]].key_idx == slot) j++;
            for (uint32_t b = i; b < j; b += per)
                sl.h_work[items++] = WorkItem{slot, b, std::min(per, j - b), ctx->h_keys[slot].nr};
            keys++;
            i = j;
        }
        std::copy(ord.begin(), ord.end(), sl.h_perm);
        *sl.h_nwork = items;
        HIP_TRY(ctx, launch_aes_gcm_burst(true, ctx->d_keys, descs, sl.v_plan, (uint32_t)ord.size(), keys, per,
                                          q->v_ring, nullptr, nullptr, QPP_HP_APPLY, q->suites & kAesSuites, ctx->pow,
                                          s));
    }
    if (q->suites & ~kAesSuites)
        HIP_TRY(ctx, launch_chacha(true, ctx->d_keys, ctx->key_cap, descs, n, q->v_ring, nullptr, nullptr,
                                   QPP_HP_APPLY, true, s));
    return QPP_OK;
}

// the slot's last flush is over (host wait); its buffers may be refilled
static int txq_slot_drain(qpp_txq *q, TxqSlot &sl) {
    if (!sl.busy) return QPP_OK;
    HIP_TRY(q->ctx, hipEventSynchronize(sl.done));
    sl.busy = false;
    return QPP_OK;
}
// A completed flush whose packets the FIPS nonce-order gate refused (left unsealed in the ring) reports
// QPP_INTERNAL_ERROR once: to the first wait / poll of one of its tickets, or else to the flush that reuses its slot.
static int txq_refused(TxqSlot &sl) {
    if (!*sl.h_refused) return QPP_OK;
    *sl.h_refused = 0;
    return QPP_INTERNAL_ERROR;
}

// The pushed batch is handed over: the next pushes start a new one
static void txq_reset_batch(qpp_txq *q) {
    q->pend_first = q->pend_last = 0;
    q->pend_bursts = 0;
    q->count = q->count_at_ticket = 0;
    q->lo = SIZE_MAX;
    q->hi = 0;
    q->suites = 0;
}

// Persistent queue: posts slots[cur]'s packets (any suite, no FIPS key live) to the server.  The descriptors are copied
// into the server's plan (key-sorted, items of <= one packet per wave), so the slot is free for the next pushes at
// once; the previous posted flush must be done first (its plan is being rewritten).
// Before a post: the previous one done, key records installed since visible to the server (and a new key epoch), the
// server on the current key table and not possibly leaving on its idle timeout
static int srv_prepare(qpp_txq *q, std::chrono::steady_clock::time_point now) {
    qpp_ctx *ctx = q->ctx;
    RC_TRY(srv_wait(q, q->srv_posted));
    if (ctx->key_gen != q->srv_key_gen) {
        // records installed since the last post are in HBM before the server reads them (host wait, only after key
        // changes), and the new epoch drops every workgroup's cached GHASH tables (a slot may hold a new key now)
        HIP_TRY(ctx, hipEventSynchronize(ctx->keys_ready));
        q->srv_key_gen = ctx->key_gen;
        q->srv_epoch = (q->srv_epoch + 1u) & 0xffu;
    }
    // a one-shot launch that served the last flush has left before anything is posted again (it would serve it too)
    if (q->oneshot_ev) HIP_TRY(ctx, hipEventSynchronize(q->oneshot_ev));
    if (q->srv_running && q->srv_keys != ctx->d_keys) RC_TRY(srv_stop(q));  // (grow_keys stops servers already)
    // a server idle for long may be leaving on its own timeout: never post to it (part of it could miss the flush)
    if (q->srv_running && now - q->srv_last_post > q->srv_host_idle) RC_TRY(srv_stop(q));
    return QPP_OK;
}

// (the caller ran srv_prepare and started the server)
static int srv_submit(qpp_txq *q, std::chrono::steady_clock::time_point now) {
    qpp_ctx *ctx = q->ctx;
    TxqSlot &sl = q->slots[q->cur];
    const uint32_t n = (uint32_t)q->count;
    const uint32_t W = kTxsWaves;
    std::vector<uint32_t> &ord = q->order;
    ord.resize(n);
    bool one_key = true;  // (the usual GSO burst: one connection's key; no sort then)
    for (uint32_t i = 0; i < n; i++) {
        ord[i] = i;
        one_key = one_key && sl.h_desc[i].key_idx == sl.h_desc[0].key_idx;
    }
    if (!one_key)
        std::stable_sort(ord.begin(), ord.end(),
                         [&sl](uint32_t a, uint32_t b) { return sl.h_desc[a].key_idx < sl.h_desc[b].key_idx; });
    // packets per item: spread the flush over the server's workgroups, at most one packet per wave
    const uint32_t per = std::max(1u, std::min(W, (n + q->srv_wgs - 1) / q->srv_wgs));
    uint32_t items = 0;
    for (uint32_t i = 0; i < n;) {
        const uint32_t slot = sl.h_desc[ord[i]].key_idx;
        uint32_t j = i;
        while (j < n && sl.h_desc[ord[j]].key_idx == slot) j++;
        for (uint32_t b = i; b < j; b += per) {
            const uint32_t cnt = std::min(per, j - b);
            q->h_items[items] = WorkItem{slot, items * W, cnt, ctx->h_keys[slot].nr};
            for (uint32_t k = 0; k < cnt; k++) q->h_sdesc[(size_t)items * W + k] = sl.h_desc[ord[b + k]];
            items++;
        }
        i = j;
    }
    q->srv_seq = srv_next(q->srv_seq);
    const uint32_t seq = q->srv_seq, word = (q->srv_epoch << 24) | items;
    // each workgroup's slot: its first item and that item's descriptors, every 16-byte chunk tagged, then the seq (x86
    // stores are seen in order; the server reads each chunk in one load and checks every tag, so a read that raced
    // these stores is repeated)
    for (uint32_t b = 0; b < q->srv_wgs; b++) {
        TxsSlot &sl = q->h_slots[b];
        sl.word = word;
        const WorkItem it = b < items ? q->h_items[b] : WorkItem{0, 0, 0, 0};
        for (uint32_t k = 0; k < it.count; k++) {
            const qpp_pkt &d = q->h_sdesc[(size_t)b * W + k];
            TxsSlotDesc &sd = sl.desc[k];
            sd.pn = d.pn;
            sd.key_idx = d.key_idx;
            __atomic_store_n(&sd.tag0, seq, __ATOMIC_RELEASE);  // (after the chunk's other words)
            sd.off = d.off;
            sd.lens = (uint32_t)d.aad_len | (uint32_t)d.pt_len << 16;
            sd.misc = (uint32_t)d.pn_len | (uint32_t)d.flags << 8;
            __atomic_store_n(&sd.tag1, seq, __ATOMIC_RELEASE);
        }
        sl.it_key = it.key;
        sl.it_count = it.count;
        sl.it_nr = it.nr;
        __atomic_store_n(&sl.it_tag, seq, __ATOMIC_RELEASE);
        __atomic_store_n(&sl.seq, seq, __ATOMIC_RELEASE);
    }
    q->srv_last_post = now;
    q->srv_posted = q->srv_seq;
    q->srv_first = q->pend_first;
    q->srv_last = q->pend_last;
    q->n_server++;
    txq_reset_batch(q);
    return QPP_OK;
}

// Sends slots[cur] (every burst flushed into it) and moves on to the next slot, once that one's last flush is over.
static int txq_submit(qpp_txq *q) {
    if (!q->pend_bursts) return QPP_OK;
    qpp_ctx *ctx = q->ctx;
    HIP_TRY(ctx, hipSetDevice(ctx->device));
    RC_TRY(flush_keys(ctx));
    if (q->persistent) {
        if (!ctx->fips_live) {
            const auto now = std::chrono::steady_clock::now();
            RC_TRY(srv_prepare(q, now));
            const int rc = srv_start(q);
            if (rc != kNoServerSlot) {
                RC_TRY(rc);
                return srv_submit(q, now);
            }
            // every server slot of the device is taken: this flush is launched (the same bytes)
        }
        // FIPS gating takes the launched path (its nonce-order gate), behind the posted flush
        RC_TRY(srv_wait(q, q->srv_posted));
    }
    q->n_launch++;
    TxqSlot &sl = q->slots[q->cur];
    const uint32_t n = (uint32_t)q->count;
    StreamState *st = nullptr;
    RC_TRY(batch_stream(ctx, sl.stream, &st));  // sees the latest key install
    const bool gate = ctx->fips_live > 0;
    if (gate) {
        RC_TRY(ensure_fips(ctx, st, n));
        HIP_TRY(ctx, hipMemsetAsync(st->fips_refused, 0, 4, sl.stream));
    }
    if (n <= q->zc_max) {
        RC_TRY(txq_enqueue_zero_copy(q, sl, st, n));
    } else {
        hipStream_t s = sl.stream;
        // Only this flush's own packet bytes travel, as runs of adjacent packets: the ring between and around them
        // belongs to the transport or to other flushes in flight (a copy of the whole [lo, hi) span would write stale
        // device bytes over them on the way back)
        std::vector<std::pair<size_t, size_t>> &runs = q->runs;
        runs.clear();
        for (uint32_t i = 0; i < n; i++) {
            const qpp_pkt &d = sl.h_desc[i];
            runs.emplace_back((size_t)d.off, (size_t)d.off + d.aad_len + d.pt_len + 16);
        }
        std::sort(runs.begin(), runs.end());
        size_t w = 0;
        for (size_t i = 1; i < runs.size(); i++) {
            if (runs[i].first <= runs[w].second) runs[w].second = std::max(runs[w].second, runs[i].second);
            else runs[++w] = runs[i];
        }
        runs.resize(w + 1);
        for (const auto &r : runs)
            HIP_TRY(ctx, hipMemcpyAsync(q->d_ring + r.first, q->h_ring + r.first, r.second - r.first,
                                        hipMemcpyHostToDevice, s));
        HIP_TRY(ctx, hipMemcpyAsync(sl.d_desc, sl.h_desc, sizeof(qpp_pkt) * n, hipMemcpyHostToDevice, s));
        uint32_t flags = QPP_HP_APPLY;
        if (!(q->suites & ~kAesSuites)) flags |= QPP_ONLY_AES;
        else if (!(q->suites & kAesSuites)) flags |= QPP_ONLY_CHACHA;
        RC_TRY(enqueue_seal(ctx, st, sl.d_desc, n, q->d_ring, nullptr, nullptr, flags, st->fips_refused));
        for (const auto &r : runs)
            HIP_TRY(ctx, hipMemcpyAsync(q->h_ring + r.first, q->d_ring + r.first, r.second - r.first,
                                        hipMemcpyDeviceToHost, s));
    }
    if (gate) HIP_TRY(ctx, hipMemcpyAsync(sl.h_refused, st->fips_refused, 4, hipMemcpyDeviceToHost, sl.stream));
    RC_TRY(note_work(ctx, st));  // key retirement orders behind this flush
    HIP_TRY(ctx, hipEventRecord(sl.done, sl.stream));
    sl.busy = true;
    sl.first = q->pend_first;
    sl.last = q->pend_last;
    txq_reset_batch(q);
    // the next batch fills the next slot, once that slot's previous flush is over (back-pressure)
    q->cur = (q->cur + 1) % q->slots.size();
    RC_TRY(txq_slot_drain(q, q->slots[q->cur]));
    return txq_refused(q->slots[q->cur]);
}

int qpp_txq_set_coalesce(qpp_txq *q, size_t bursts) {
    if (!q || !bursts || bursts > 1024) return QPP_INTERNAL_ERROR;
    q->coalesce = (uint32_t)bursts;
    return QPP_OK;
}

int qpp_txq_flush_async(qpp_txq *q, uint64_t *ticket) {
    if (!q || !ticket) return QPP_INTERNAL_ERROR;
    *ticket = 0;
    const size_t burst = q->count - q->count_at_ticket;
    if (!burst) return QPP_OK;  // nothing pushed since the last flush: ticket 0 is always complete
    *ticket = q->next_ticket++;
    if (!q->pend_first) q->pend_first = *ticket;
    q->pend_last = *ticket;
    q->pend_bursts++;
    q->count_at_ticket = q->count;
    // send now once `coalesce` bursts are in, or when another burst of this size would not fit the slot
    if (q->pend_bursts >= q->coalesce || q->count + burst > q->max_packets) return txq_submit(q);
    return QPP_OK;
}

// the slot holding `ticket` (submitting it first if it is still being coalesced); nullptr: long complete
static int txq_slot_of(qpp_txq *q, uint64_t ticket, TxqSlot **out) {
    *out = nullptr;
    if (!ticket) return QPP_OK;
    if (q->pend_first && ticket >= q->pend_first && ticket <= q->pend_last) RC_TRY(txq_submit(q));
    for (TxqSlot &sl : q->slots)
        if (sl.first && ticket >= sl.first && ticket <= sl.last) { *out = &sl; break; }
    return QPP_OK;
}

// a ticket of the flush last posted to the server (earlier posted ones are done: one is posted at a time)
static bool srv_ticket(const qpp_txq *q, uint64_t ticket) {
    return q->persistent && q->srv_first && ticket >= q->srv_first && ticket <= q->srv_last;
}

int qpp_txq_poll(qpp_txq *q, uint64_t ticket, int *done) {
    if (!q || !done) return QPP_INTERNAL_ERROR;
    if (ticket >= q->next_ticket) return QPP_INTERNAL_ERROR;
    TxqSlot *sl = nullptr;
    RC_TRY(txq_slot_of(q, ticket, &sl));
    if (srv_ticket(q, ticket)) {
        *done = srv_done(q, q->srv_posted);
        if (!*done && !srv_alive(q)) RC_TRY(srv_start(q));
        return QPP_OK;
    }
    if (!sl) { *done = 1; return QPP_OK; }
    if (!sl->busy) { *done = 1; return txq_refused(*sl); }
    const hipError_t e = hipEventQuery(sl->done);
    if (e == hipErrorNotReady) { *done = 0; return QPP_OK; }
    HIP_TRY(q->ctx, e);
    sl->busy = false;
    *done = 1;
    return txq_refused(*sl);
}

int qpp_txq_wait(qpp_txq *q, uint64_t ticket) {
    if (!q) return QPP_INTERNAL_ERROR;
    if (ticket >= q->next_ticket) return QPP_INTERNAL_ERROR;
    TxqSlot *sl = nullptr;
    RC_TRY(txq_slot_of(q, ticket, &sl));
    if (srv_ticket(q, ticket)) return srv_wait(q, q->srv_posted);
    if (!sl) return QPP_OK;
    RC_TRY(txq_slot_drain(q, *sl));
    return txq_refused(*sl);
}

}  // extern "C"

// A queue with a persistent server of `wgs` workgroups.  Fine-grained (coherent) pinned memory for everything the
// server touches: polled over PCIe while the host writes it, and read and written by a kernel that does not end
// between flushes (no cached copy may outlive a flush) -- the ring too.
static int txq_create_server(qpp_ctx *ctx, size_t ring_bytes, size_t max_packets, uint32_t wgs, uint32_t idle_ms,
                             qpp_txq **out) {
    if (!ctx || !out || max_packets >= kTxsItemsMask) return QPP_INTERNAL_ERROR;
    const unsigned fl = hipHostMallocCoherent | hipHostMallocMapped;
    RC_TRY(txq_create(ctx, ring_bytes, max_packets, 1, fl, out));
    qpp_txq *q = *out;
    auto bad = [&](hipError_t e, const char *what) {
        if (!fail(ctx, e, what)) return false;
        qpp_txq_destroy(q);
        *out = nullptr;
        return true;
    };
    q->persistent = true;
    ctx->servers.push_back(q);
    hipError_t ev_err = hipSuccess;
    {
        DevServers &r = dev_servers(ctx->device);
        std::lock_guard<std::mutex> lk(r.mu);
        if (!r.h_evict) {  // (process lifetime: one 16-B word per device, never freed)
            void *h = nullptr, *dv = nullptr;
            ev_err = hipHostMalloc(&h, 16, fl);
            if (ev_err == hipSuccess) ev_err = hipHostGetDevicePointer(&dv, h, 0);
            if (ev_err == hipSuccess) {
                memset(h, 0, 16);
                r.h_evict = (uint32_t *)h;
                r.v_evict = (uint32_t *)dv;
            }
        }
        r.queues.push_back(q);
    }
    if (bad(ev_err, "eviction word")) return QPP_DEVICE_ERROR;
    const size_t W = kTxsWaves;
    void *v = nullptr;
    if (bad(hmalloc(&q->h_mail, sizeof(TxsMail), fl), "txq server mailbox") ||
        bad(hipHostGetDevicePointer(&v, q->h_mail, 0), "mailbox view"))
        return QPP_DEVICE_ERROR;
    q->v_mail = (TxsMail *)v;
    memset(q->h_mail, 0, sizeof(TxsMail));
    if (bad(hmalloc(&q->h_items, sizeof(WorkItem) * max_packets, fl), "txq server items") ||
        bad(hipHostGetDevicePointer(&v, q->h_items, 0), "items view"))
        return QPP_DEVICE_ERROR;
    q->v_items = (WorkItem *)v;
    if (bad(hmalloc(&q->h_sdesc, sizeof(qpp_pkt) * max_packets * W, fl), "txq server descs") ||
        bad(hipHostGetDevicePointer(&v, q->h_sdesc, 0), "descs view"))
        return QPP_DEVICE_ERROR;
    q->v_sdesc = (qpp_pkt *)v;
    memset(q->h_sdesc, 0, sizeof(qpp_pkt) * max_packets * W);
    // The server's stream at the device's greatest priority: the runtime maps streams onto at most GPU_MAX_HW_QUEUES
    // hardware queues per priority level, round-robin, and a kernel queued behind a persistent one on the same hardware
    // queue waits for its idle exit -- found by tests/test_gpu_txrx.py: after another context's streams had come and
    // gone, the context's batch stream shared the server's queue and its seal started 30 s late.  A priority level of
    // its own keeps the servers off the batch streams' queues (at most GPU_MAX_HW_QUEUES servers per process).
    int prio_least = 0, prio_greatest = 0;
    if (bad(hipDeviceGetStreamPriorityRange(&prio_least, &prio_greatest), "stream priorities") ||
        bad(hipStreamCreateWithPriority(&q->srv_stream, hipStreamNonBlocking, prio_greatest), "txq server stream"))
        return QPP_DEVICE_ERROR;
    q->srv_wgs = std::max(1u, std::min(wgs, ctx->n_cu));
    if (bad(hmalloc(&q->h_slots, sizeof(TxsSlot) * q->srv_wgs, fl), "txq server slots") ||
        bad(hipHostGetDevicePointer(&v, q->h_slots, 0), "slots view"))
        return QPP_DEVICE_ERROR;
    q->v_slots = (TxsSlot *)v;
    memset(q->h_slots, 0, sizeof(TxsSlot) * q->srv_wgs);
    idle_ms = std::min<uint32_t>(std::max(4u, idle_ms), 40000u);
    q->srv_idle_ticks = idle_ms * 100000u;  // s_memrealtime: 100 MHz
    q->srv_host_idle = std::chrono::microseconds(250u * idle_ms);
    return QPP_OK;
}

static uint32_t srv_idle_ms() {
    const char *e = getenv("QPP_TXQ_SERVER_IDLE_MS");
    return e ? (uint32_t)strtoul(e, nullptr, 10) : 200u;
}

extern "C" {

int qpp_txq_create_persistent(qpp_ctx *ctx, size_t ring_bytes, size_t max_packets, qpp_txq **out) {
    uint32_t wgs = 16;
    if (const char *e = getenv("QPP_TXQ_SERVER_WGS")) wgs = (uint32_t)strtoul(e, nullptr, 10);
    return txq_create_server(ctx, ring_bytes, max_packets, wgs, srv_idle_ms(), out);
}

int qpp_txq_server_refused(const qpp_txq *q, uint64_t *count) {
    if (!q || !count || !q->persistent) return QPP_INTERNAL_ERROR;
    *count = __atomic_load_n(&q->h_mail->oob, __ATOMIC_ACQUIRE);
    return QPP_OK;
}

int qpp_txq_server_time(const qpp_txq *q, double *us) {
    if (!q || !us || !q->persistent) return QPP_INTERNAL_ERROR;
    *us = (double)(q->h_mail->t_done - q->h_mail->t_seen) / 100.0;
    return QPP_OK;
}

int qpp_txq_server_stamps(const qpp_txq *q, uint64_t out[12]) {
    if (!q || !out || !q->persistent) return QPP_INTERNAL_ERROR;
    const TxsMail &m = *q->h_mail;
    const uint64_t v[12] = {m.t_seen, m.pad0[0], m.pad0[1], m.pad0[2], m.pad0[3], m.t_done, m.pad0[4],
                            m.pad1[0], m.pad1[1], m.pad1[2], m.pad1[3], m.pad1[4]};
    memcpy(out, v, sizeof v);
    return QPP_OK;
}

int qpp_txq_info(const qpp_txq *q, uint64_t *server_flushes, uint64_t *launched_flushes, uint64_t *server_starts) {
    if (!q) return QPP_INTERNAL_ERROR;
    if (server_flushes) *server_flushes = q->n_server;
    if (launched_flushes) *launched_flushes = q->n_launch;
    if (server_starts) *server_starts = q->n_starts;
    return QPP_OK;
}

int qpp_dev_server_evictions(int device, uint64_t *evictions, uint64_t *oneshots) {
    if (device < 0 || device >= 64) return QPP_INTERNAL_ERROR;
    DevServers &r = dev_servers(device);
    std::lock_guard<std::mutex> lk(r.mu);
    if (evictions) *evictions = r.evictions;
    if (oneshots) *oneshots = r.oneshots;
    return QPP_OK;
}

int qpp_txq_flush(qpp_txq *q) {
    uint64_t t = 0;
    RC_TRY(qpp_txq_flush_async(q, &t));
    return qpp_txq_wait(q, t);
}

}  // extern "C"

namespace {

// Key::encrypt / Key::decrypt (crypto/src/packet_protection.rs; cipher_suite.rs:86-160) of one packet through the
// context's packet server: the header and payload (and the tag, to open) are copied into its pinned ring, posted as
// one work item to workgroup slot % kPktWgs (so a connection's sealer and opener keep their GHASH tables in different
// workgroups' LDS), sealed without header protection or opened in place there, and copied back.  No launch, no
// runtime call: the cost is the post's PCIe round trip, the packet's own read / AES / GHASH / write chain and the copies.
constexpr size_t kPktRing = 16384;  // header + payload + tag; longer packets take the launched path
// zeroes the packet server's ring bytes of a call on every exit path (an early return left plaintext there)
struct RingWipe {
    uint8_t *p;
    size_t n;
    ~RingWipe() { secure_zero(p, n); }
};
constexpr uint32_t kPktWgs = 4;

// Posts one work item of one packet (ring offset 0) to workgroup wg of the packet server -- every other workgroup an
// empty item -- and waits for it.  The slot's status byte is preset to INTERNAL_ERROR (left so if the record is not
// what the item names).
int srv_post_one(qpp_txq *q, std::chrono::steady_clock::time_point now, uint32_t wg, uint32_t slot, uint32_t nr,
                 uint64_t pn, uint32_t lens, uint32_t misc) {
    RC_TRY(srv_start(q, true));  // (the caller found it a server slot)
    q->srv_seq = srv_next(q->srv_seq);
    const uint32_t seq = q->srv_seq;
    const uint32_t word = (q->srv_epoch << 24) | q->srv_wgs;  // item b for workgroup b; all but one empty
    for (uint32_t b = 0; b < q->srv_wgs; b++) {
        TxsSlot &sl = q->h_slots[b];
        sl.word = word;
        if (b == wg) {
            sl.status[0] = (int8_t)QPP_INTERNAL_ERROR;
            TxsSlotDesc &sd = sl.desc[0];
            sd.pn = pn;
            sd.key_idx = slot;
            __atomic_store_n(&sd.tag0, seq, __ATOMIC_RELEASE);
            sd.off = 0;
            sd.lens = lens;
            sd.misc = misc;
            __atomic_store_n(&sd.tag1, seq, __ATOMIC_RELEASE);
        }
        sl.it_key = b == wg ? slot : 0u;
        sl.it_count = b == wg ? 1u : 0u;
        sl.it_nr = b == wg ? nr : 0u;
        __atomic_store_n(&sl.it_tag, seq, __ATOMIC_RELEASE);
        __atomic_store_n(&sl.seq, seq, __ATOMIC_RELEASE);
    }
    q->srv_last_post = now;
    q->srv_posted = seq;
    q->srv_first = q->srv_last = 0;  // (no ticket: nothing of the transmit-queue API refers to this post)
    q->n_server++;
    q->ctx->pkt_calls++;
    return srv_wait(q, seq);
}

int packet_server_get(qpp_ctx *ctx, qpp_txq **out) {
    if (!ctx->pkt_q) RC_TRY(txq_create_server(ctx, kPktRing, 1, kPktWgs, srv_idle_ms(), &ctx->pkt_q));
    *out = ctx->pkt_q;
    return QPP_OK;
}
int packet_server_run(const qpp_key *k, bool seal, uint64_t pn, const uint8_t *header, size_t header_len,
                      const uint8_t *payload, size_t payload_len, uint8_t *out, uint8_t *tag_out, int8_t *status_out,
                      bool *handled) {
    qpp_ctx *ctx = k->ctx;
    *handled = false;
    const DevKey &rec = ctx->h_keys[k->slot];
    const size_t total = header_len + payload_len + 16;
    // FIPS seals keep the launched path (its nonce-order gate)
    if (!ctx->pkt_server || (seal && rec.fips) || total > kPktRing) return QPP_OK;
    qpp_txq *q = nullptr;
    RC_TRY(packet_server_get(ctx, &q));
    RC_TRY(flush_keys(ctx));
    const auto now = std::chrono::steady_clock::now();
    RC_TRY(srv_prepare(q, now));
    const int rc = srv_start(q);
    if (rc == kNoServerSlot) return QPP_OK;  // every server slot of the device is taken: the caller launches it
    RC_TRY(rc);
    uint8_t *r = q->h_ring;
    RingWipe wipe{r, total};  // the plaintext never stays in the host-visible ring, whatever the exit path
    if (header_len) memcpy(r, header, header_len);
    if (payload_len) memcpy(r + header_len, payload, payload_len);
    if (!seal) memcpy(r + header_len + payload_len, tag_out, 16);
    const uint32_t wg = k->slot % q->srv_wgs;
    RC_TRY(srv_post_one(q, now, wg, k->slot, rec.nr, pn, (uint32_t)header_len | (uint32_t)payload_len << 16,
                        (uint32_t)(seal ? kTxsPktNoHp : kTxsPktOpen) << 8));
    *status_out = __atomic_load_n(&q->h_slots[wg].status[0], __ATOMIC_ACQUIRE);
    *handled = true;
    if (!(seal && *status_out != QPP_OK)) {  // (a refused seal leaves the caller's buffer untouched)
        memcpy(out, r + header_len, payload_len);
        if (seal) memcpy(tag_out, r + header_len + payload_len, 16);
    }
    return QPP_OK;
}

}  // namespace

namespace {

// HeaderKey::*_header_protection_mask of one sample (header_key.rs:52-56) through the packet server: the sample at
// ring offset 0, the mask written at 16 by a mask item (kTxsMaskNr) on workgroup slot % kPktWgs
int packet_server_mask(qpp_ctx *ctx, uint32_t slot, const uint8_t *sample, uint8_t mask[5], bool *handled) {
    *handled = false;
    if (!ctx->pkt_server || slot >= ctx->key_cap || !ctx->h_keys[slot].live) return QPP_OK;
    qpp_txq *q = nullptr;
    RC_TRY(packet_server_get(ctx, &q));
    RC_TRY(flush_keys(ctx));
    const auto now = std::chrono::steady_clock::now();
    RC_TRY(srv_prepare(q, now));
    const int rc = srv_start(q);
    if (rc == kNoServerSlot) return QPP_OK;  // every server slot of the device is taken: the caller launches it
    RC_TRY(rc);
    uint8_t *r = q->h_ring;
    RingWipe wipe{r, 32};
    memcpy(r, sample, 16);
    memset(r + 16, 0, 16);
    RC_TRY(srv_post_one(q, now, slot % q->srv_wgs, slot, kTxsMaskNr, 0, 16, 0));
    memcpy(mask, r + 16, 5);
    *handled = true;
    return QPP_OK;
}

}  // namespace

extern "C" {

int qpp_ctx_set_packet_server(qpp_ctx *ctx, int on) {
    if (!ctx) return QPP_INTERNAL_ERROR;
    ctx->pkt_server = on != 0;
    if (!on && ctx->pkt_q) {
        HIP_TRY(ctx, hipSetDevice(ctx->device));
        ctx->pkt_starts += ctx->pkt_q->n_starts;
        qpp_txq_destroy(ctx->pkt_q);
        ctx->pkt_q = nullptr;
    }
    return QPP_OK;
}

int qpp_ctx_packet_server_info(const qpp_ctx *ctx, uint64_t *calls, uint64_t *starts) {
    if (!ctx) return QPP_INTERNAL_ERROR;
    if (calls) *calls = ctx->pkt_calls;
    if (starts) *starts = ctx->pkt_starts + (ctx->pkt_q ? ctx->pkt_q->n_starts : 0);
    return QPP_OK;
}

}  // extern "C"
