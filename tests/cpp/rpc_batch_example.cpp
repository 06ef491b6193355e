// rpc_batch_example.cpp -- the receive path of Photon's RPC with batched
// checksum validation, in plain C++ against the public headers:
//  * payload buffers come from the pinned IOAlloc callbacks
//    (photon_crc_pinned_allocate / _deallocate, common/io-alloc.h:31-85);
//  * the sender computes CheckedMessage::add_checksum as the reference does
//    (rpc/serialize.h:239-261, 425): the drop-in crc32c_extend chained over
//    the payload, accumulating IN PLACE in m_checksum -- the first 4 bytes of
//    the message struct (its CheckedMessage<> base) -- then over the struct
//    holding that running value;
//  * the receiver does what validate_checksum does (serialize.h:266-275,
//    462-463) -- save m_checksum, zero it -- but adds the message to a batch
//    and checks all of them with one GPU submit. Struct fields corrupted in
//    flight are rejected; payload corrupted in flight is accepted, exactly as
//    Photon's own validate_checksum accepts it (the in-place accumulation
//    cancels the payload's CRC). A DETACHED_BODY batch over the
//    same messages (payload hashed, then the struct with m_checksum = 0)
//    catches both.
// Exit 0 iff every verdict is right.
#include <photon/common/checksum/crc32c.h>
#include <photon_crc/checked_batch.h>

#include <stdio.h>
#include <string.h>

#include <atomic>
#include <random>
#include <vector>

struct RequestStruct {  // a Photon message struct: CheckedMessage<> base first
    uint32_t m_checksum;
    uint32_t fields[9];
    uint64_t seq;
};

struct Received {
    std::vector<photon_crc_iovec> iov;
    RequestStruct* msg;
};

int main() {
    const int kMsgs = 4096, kSegs = 8, kSegLen = 8192;
    if (photon_crc_device_count() <= 0) {
        fprintf(stderr, "no device: %s\n", photon_crc_last_error());
        return 2;
    }
    std::mt19937_64 rng(42);
    std::vector<void*> blocks;
    std::vector<Received> rx(kMsgs);
    for (int m = 0; m < kMsgs; ++m) {
        uint32_t crc = 0;  // Crc32Hasher::init_value()
        for (int s = 0; s < kSegs; ++s) {
            void* p = nullptr;
            const int len = kSegLen - (int)(rng() % 64);
            if (photon_crc_pinned_allocate(nullptr, photon_crc_range{len, len}, &p) != len) return 3;
            blocks.push_back(p);
            auto* b = static_cast<uint8_t*>(p);
            for (int k = 0; k < len; ++k) b[k] = (uint8_t)rng();
            rx[m].iov.push_back({p, (uint64_t)len});
            crc = crc32c_extend(p, len, crc);
        }
        void* sp = nullptr;
        if (photon_crc_pinned_allocate(nullptr, photon_crc_range{(int)sizeof(RequestStruct), (int)sizeof(RequestStruct)},
                                       &sp) <= 0)
            return 3;
        blocks.push_back(sp);
        auto* req = static_cast<RequestStruct*>(sp);
        req->seq = m;
        for (auto& f : req->fields) f = (uint32_t)rng();
        // add_checksum: m_checksum IS the accumulator (Crc32Hasher::extend_hash
        // takes it by reference), so the struct is hashed holding the running CRC
        req->m_checksum = crc;
        req->m_checksum = crc32c_extend(req, sizeof(*req), req->m_checksum);
        rx[m].msg = req;
    }
    // in flight: every 97th message gets a struct field flipped, every 89th a payload byte
    for (int m = 0; m < kMsgs; m += 97) rx[m].msg->fields[3] ^= 0x10;
    for (int m = 0; m < kMsgs; m += 89) static_cast<uint8_t*>(const_cast<void*>(rx[m].iov[2].base))[100] ^= 0x10;

    photon_crc_msg_batch* batch = photon_crc_msg_batch_create(kMsgs, kMsgs * (kSegs + 1), 0);
    if (!batch) return 4;
    for (int m = 0; m < kMsgs; ++m) {
        const uint32_t dst = rx[m].msg->m_checksum;  // validate_checksum: save, zero, re-hash
        rx[m].msg->m_checksum = 0;
        if (photon_crc_msg_batch_add(batch, rx[m].iov.data(), kSegs, rx[m].msg, sizeof(RequestStruct), dst) != m)
            return 5;
    }
    std::atomic<int> signalled{0};
    if (photon_crc_msg_batch_submit(batch, nullptr, [](void* a) { static_cast<std::atomic<int>*>(a)->store(1); },
                                    &signalled))
        return 6;
    const int64_t bad = photon_crc_msg_batch_wait(batch);
    int wrong = 0;
    for (int m = 0; m < kMsgs; ++m) {
        const int v = photon_crc_msg_batch_result(batch, m, nullptr);
        if (v != (m % 97 ? 1 : 0)) ++wrong;  // struct corruption rejected, payload corruption accepted (= Photon)
    }
    const int expect_bad = (kMsgs + 96) / 97;
    // DETACHED_BODY: payload + struct (m_checksum = 0); its value differs from
    // Photon's, so compare with the same chain recomputed on the host engine.
    photon_crc_msg_batch* det = photon_crc_msg_batch_create(kMsgs, kMsgs * (kSegs + 1), PHOTON_CRC_BATCH_DETACHED_BODY);
    if (!det) return 7;
    std::vector<uint32_t> chain(kMsgs);
    for (int m = 0; m < kMsgs; ++m) {
        uint32_t c = 0;
        for (auto& v : rx[m].iov) c = crc32c_extend(v.base, v.len, c);
        chain[m] = crc32c_extend(rx[m].msg, sizeof(RequestStruct), c);
        if (photon_crc_msg_batch_add(det, rx[m].iov.data(), kSegs, rx[m].msg, sizeof(RequestStruct), chain[m]) != m)
            return 8;
    }
    if (photon_crc_msg_batch_submit(det, nullptr, nullptr, nullptr) || photon_crc_msg_batch_wait(det) != 0) ++wrong;
    photon_crc_msg_batch_destroy(det);
    printf("rpc_batch_example: %d messages, %lld rejected (expected %d: struct corruption; payload corruption passes "
           "as in Photon), %d wrong verdicts, callback %d\n",
           kMsgs, (long long)bad, expect_bad, wrong, signalled.load());
    photon_crc_msg_batch_destroy(batch);
    for (void* p : blocks) photon_crc_pinned_deallocate(nullptr, p);
    return (bad == expect_bad && !wrong && signalled.load() == 1) ? 0 : 1;
}
