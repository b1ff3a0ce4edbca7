/* txqdrive.c — native driver loop for `bench.py --mode txq --inflight K` (the transport's side of qpp_txq, in C so
 * that the bench measures the engine and not Python's per-call cost).  Per burst: wait for the ring region's previous
 * ticket, push `burst` ready descriptors (one qpp_txq_push_descs), qpp_txq_flush_async.  Build: see Makefile.
 *
 *   double txq_drive(qpp_txq *q, const qpp_pkt *proto, size_t burst, size_t region_bytes, size_t regions,
 *                    size_t bursts, uint64_t pn0)  -> seconds for `bursts` bursts (all waited for), < 0 on error
 *   int txq_latency(qpp_txq *q, const qpp_pkt *proto, size_t burst, size_t bursts, uint64_t pn0, double *lat_us)
 *        -> one burst at a time: push, then qpp_txq_flush (seal and wait); lat_us[k] = that call's duration
 *   int rotate_keys(qpp_ctx *ctx, qpp_key **keys, size_t n, uint32_t *slots)
 *        -> a KeySet rotation of every connection (BASELINE configs[4]): keys[i] <- its next-phase key
 *           (qpp_key_update_batch), the old keys freed (qpp_key_free_batch), slots[i] = the new slots, and the
 *           connection table repointed (qpp_ctx_set_conn_keys), as the transport would call it
 *   int packet_latency(qpp_key *k, const uint8_t *header, size_t header_len, const uint8_t *payload,
 *                      size_t payload_len, size_t calls, uint64_t pn0, double *seal_us, double *open_us,
 *                      double *mask_us)
 *        -> Key::encrypt, the sealing HeaderKey mask of a sample of the sealed packet, then Key::decrypt of one packet
 *           per call (qpp_seal, qpp_hp_mask, qpp_open), each call timed; the opened bytes checked against the payload
 *           (returns -5 on a mismatch)
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "../include/qpp.h"

static double now_s(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (double)t.tv_sec + 1e-9 * (double)t.tv_nsec;
}

double txq_drive(qpp_txq *q, const qpp_pkt *proto, size_t burst, size_t region_bytes, size_t regions, size_t bursts,
                 uint64_t pn0) {
    qpp_pkt *d = (qpp_pkt *)malloc(sizeof(qpp_pkt) * burst);
    uint64_t *tickets = (uint64_t *)calloc(regions, sizeof(uint64_t));
    if (!d || !tickets) return -1.0;
    uint64_t pn = pn0;
    const double t0 = now_s();
    for (size_t k = 0; k < bursts; k++) {
        const size_t r = k % regions;
        if (qpp_txq_wait(q, tickets[r]) != QPP_OK) return -2.0;  /* the region's previous burst is sent */
        memcpy(d, proto, sizeof(qpp_pkt) * burst);
        for (size_t i = 0; i < burst; i++) {
            d[i].pn = pn++;
            d[i].off += (uint32_t)(r * region_bytes);
        }
        if (qpp_txq_push_descs(q, d, burst) != QPP_OK) return -3.0;
        if (qpp_txq_flush_async(q, &tickets[r]) != QPP_OK) return -4.0;
    }
    for (size_t r = 0; r < regions; r++)
        if (qpp_txq_wait(q, tickets[r]) != QPP_OK) return -5.0;
    const double t = now_s() - t0;
    free(d);
    free(tickets);
    return t;
}

int txq_latency(qpp_txq *q, const qpp_pkt *proto, size_t burst, size_t bursts, uint64_t pn0, double *lat_us) {
    qpp_pkt *d = (qpp_pkt *)malloc(sizeof(qpp_pkt) * burst);
    if (!d) return -1;
    uint64_t pn = pn0;
    for (size_t k = 0; k < bursts; k++) {
        memcpy(d, proto, sizeof(qpp_pkt) * burst);
        for (size_t i = 0; i < burst; i++) d[i].pn = pn++;
        if (qpp_txq_push_descs(q, d, burst) != QPP_OK) return -3;
        const double t0 = now_s();
        if (qpp_txq_flush(q) != QPP_OK) return -4;
        lat_us[k] = 1e6 * (now_s() - t0);
    }
    free(d);
    return 0;
}

int packet_latency(qpp_key *k, const uint8_t *header, size_t header_len, const uint8_t *payload, size_t payload_len,
                   size_t calls, uint64_t pn0, double *seal_us, double *open_us, double *mask_us) {
    uint8_t *buf = (uint8_t *)malloc(payload_len + 16);
    if (!buf) return -1;
    for (size_t c = 0; c < calls; c++) {
        memcpy(buf, payload, payload_len);
        double t0 = now_s();
        if (qpp_seal(k, pn0 + c, header, header_len, buf, payload_len, payload_len + 16) != QPP_OK) return -2;
        double t1 = now_s();
        uint8_t mask[5];
        if (payload_len + 16 >= 20 && qpp_hp_mask(k, buf + 4, 16, mask) != QPP_OK) return -4;  /* sample: pn_len 0 */
        double t2 = now_s();
        if (qpp_open(k, pn0 + c, header, header_len, buf, payload_len + 16) != QPP_OK) return -3;
        double t3 = now_s();
        if (memcmp(buf, payload, payload_len) != 0) return -5;
        seal_us[c] = 1e6 * (t1 - t0);
        mask_us[c] = 1e6 * (t2 - t1);
        open_us[c] = 1e6 * (t3 - t2);
    }
    free(buf);
    return 0;
}

int rotate_keys(qpp_ctx *ctx, qpp_key **keys, size_t n, uint32_t *slots) {
    qpp_key **next = (qpp_key **)malloc(sizeof(qpp_key *) * (n ? n : 1));
    if (!next) return -1;
    int rc = qpp_key_update_batch((qpp_key *const *)keys, n, next);
    if (rc == QPP_OK) {
        qpp_key_slot_batch((const qpp_key *const *)next, n, slots);
        qpp_key_free_batch((qpp_key *const *)keys, n);
        memcpy(keys, next, sizeof(qpp_key *) * n);
        rc = qpp_ctx_set_conn_keys(ctx, slots, n);
    }
    free(next);
    return rc;
}
