// vdma_test.cpp -- the HIP vDMA target/initiator (photon_crc/vdma_hip.h) driven
// through PhotonLibOS's vDMA interface (net/vdma.h), the checks of the
// reference's net/test/test-vdma.cpp re-run against device memory, plus
// checksums of vDMA buffers against the drop-in host engine.
//
//   vdma_test local              single-process checks (test-vdma.cpp:19-147)
//   vdma_test target NAME        publish a target, fill 3 buffers, print their
//                                ids and CRCs, then serve commands on stdin
//                                ("check": CRC of buffer 2 as the target sees
//                                it; "quit")
//   vdma_test initiator NAME ID0 ID1 ID2
//                                map the ids, checksum them, overwrite buffer
//                                2 on the device and publish it with write()
// Exit 0 when every check holds; each failure prints "FAIL ...".
#include <hip/hip_runtime.h>
#include <photon/common/checksum/crc32c.h>
#include <photon_crc/crc32c_gpu.h>
#include <photon_crc/vdma_hip.h>

#include <stdio.h>
#include <string.h>

#include <atomic>
#include <iostream>
#include <string>
#include <thread>
#include <vector>

static int g_fail = 0;
#define CHECK(c)                                                  \
    do {                                                          \
        if (!(c)) {                                               \
            printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c);    \
            ++g_fail;                                             \
        }                                                         \
    } while (0)

static std::string hex(std::string_view s) {
    static const char* d = "0123456789abcdef";
    std::string h;
    for (unsigned char c : s) {
        h += d[c >> 4];
        h += d[c & 15];
    }
    return h;
}

static std::string unhex(const std::string& h) {
    std::string s;
    for (size_t i = 0; i + 1 < h.size(); i += 2) s += (char)std::stoi(h.substr(i, 2), nullptr, 16);
    return s;
}

static std::string id_of(uint64_t idx, uint64_t size) {
    uint64_t v[2] = {idx, size};
    return std::string(reinterpret_cast<const char*>(v), 16);
}

// Deterministic bytes of buffer k (a simple LCG stream).
static std::vector<uint8_t> pattern(uint32_t k, size_t n) {
    std::vector<uint8_t> v(n);
    uint64_t x = 0x9E3779B97F4A7C15ull * (k + 1);
    for (size_t i = 0; i < n; ++i) {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        v[i] = (uint8_t)(x >> 56);
    }
    return v;
}

static int local_checks() {
    const size_t unit = 4096, size = 65536;
    photon::vDMATarget* target = photon::new_hip_vdma_target(nullptr, size, unit);
    CHECK(target != nullptr);
    if (!target) return 1;

    CHECK(target->alloc(512) == nullptr);  // test-vdma.cpp:41-43
    photon::vDMABuffer* b0 = target->alloc(unit);
    photon::vDMABuffer* b1 = target->alloc(unit);
    photon::vDMABuffer* b2 = target->alloc(unit);
    CHECK(b0 && b1 && b2);
    CHECK(b0->buf_size() == unit && b1->buf_size() == unit);
    CHECK(b0->id() == id_of(0, unit) && b1->id() == id_of(1, unit) && b2->id() == id_of(2, unit));
    CHECK(b1->is_valid() && b1->is_registered());
    CHECK(b1->address() == (char*)b0->address() + unit);  // test-vdma.cpp:58,63
    CHECK(b2->address() == (char*)b1->address() + unit);
    CHECK(b0->type_code() == photon::kHipDeviceMem);

    // Buffers are device memory: fill them, checksum them in one batch.
    std::vector<std::vector<uint8_t>> host;
    photon::vDMABuffer* bufs[3] = {b0, b1, b2};
    for (int k = 0; k < 3; ++k) {
        host.push_back(pattern(k, unit));
        CHECK(hipMemcpy(bufs[k]->address(), host[k].data(), unit, hipMemcpyHostToDevice) == hipSuccess);
    }
    uint32_t crc[3] = {};
    CHECK(photon::crc32c_vdma_batch(bufs, nullptr, 3, crc) == 0);
    for (int k = 0; k < 3; ++k) CHECK(crc[k] == crc32c(host[k].data(), unit));
    const uint64_t lens[3] = {0, 1, 4095};
    CHECK(photon::crc32c_vdma_batch(bufs, lens, 3, crc) == 0);
    for (int k = 0; k < 3; ++k) CHECK(crc[k] == crc32c(host[k].data(), lens[k]));
    const uint64_t too_long[1] = {unit + 1};
    CHECK(photon::crc32c_vdma_batch(bufs, too_long, 1, crc) < 0);

    // dealloc returns the lowest index first (test-vdma.cpp:79-81 / shm.cpp:149-155).
    CHECK(target->dealloc(b0) == 0);
    photon::vDMABuffer* again = target->alloc(unit);
    CHECK(again == b0 && again->id() == id_of(0, unit));

    // Exhaustion: 16 units; the 17th alloc gives up after its retries.
    std::vector<photon::vDMABuffer*> rest;
    for (int i = 3; i < 16; ++i) rest.push_back(target->alloc(unit));
    for (auto* r : rest) CHECK(r != nullptr);
    CHECK(target->alloc(unit) == nullptr);
    for (auto* r : rest) CHECK(target->dealloc(r) == 0);
    CHECK(target->dealloc(again) == 0);
    CHECK(target->dealloc(b1) == 0);
    CHECK(target->dealloc(b2) == 0);

    // 16 threads x alloc/free: each thread always owns a distinct buffer
    // (test-vdma.cpp:117-147, OS threads instead of photon threads).
    std::atomic<int> owners[16];
    for (auto& o : owners) o = 0;
    std::atomic<int> clash{0}, nulls{0};
    std::vector<std::thread> th;
    for (int t = 0; t < 16; ++t)
        th.emplace_back([&] {
            for (int i = 0; i < 2000; ++i) {
                photon::vDMABuffer* b = target->alloc(unit);
                if (!b) {
                    ++nulls;
                    continue;
                }
                const size_t k = ((char*)b->address() - (char*)bufs[0]->address()) / unit;
                if (owners[k].fetch_add(1) != 0) ++clash;
                owners[k].fetch_sub(1);
                target->dealloc(b);
            }
        });
    for (auto& t : th) t.join();
    CHECK(clash == 0);
    CHECK(nulls == 0);

    // register_memory: host memory is pinned + mapped; device memory wrapped.
    std::vector<uint8_t> hmem = pattern(7, 1 << 20);
    photon::vDMABuffer* rh = target->register_memory(hmem.data(), hmem.size());
    CHECK(rh && rh->is_registered() && rh->address() == hmem.data() && rh->type_code() == photon::kHipRegisteredMem);
    void* dmem = nullptr;
    CHECK(hipMalloc(&dmem, 8192) == hipSuccess);
    std::vector<uint8_t> dhost = pattern(8, 8192);
    CHECK(hipMemcpy(dmem, dhost.data(), 8192, hipMemcpyHostToDevice) == hipSuccess);
    photon::vDMABuffer* rd = target->register_memory(dmem, 8192);
    CHECK(rd != nullptr);
    if (rh && rd) {
        photon::vDMABuffer* rb[2] = {rh, rd};
        uint32_t rc[2] = {};
        CHECK(photon::crc32c_vdma_batch(rb, nullptr, 2, rc) == 0);
        CHECK(rc[0] == crc32c(hmem.data(), hmem.size()));
        CHECK(rc[1] == crc32c(dhost.data(), dhost.size()));
        CHECK(target->unregister_memory(rh) == 0);
        CHECK(target->unregister_memory(rh) == -1);
        CHECK(target->unregister_memory(rd) == 0);
    }
    (void)hipFree(dmem);

    // A pageable host buffer that was never registered is refused, not read.
    std::vector<uint8_t> plain(4096, 1);
    photon::vDMABuffer* fake = nullptr;
    {
        photon::vDMATarget* t2 = photon::new_hip_vdma_target(nullptr, 4096, 4096);
        CHECK(t2 != nullptr);
        if (t2) {
            fake = t2->register_memory(plain.data(), plain.size());
            CHECK(fake != nullptr);
            CHECK(t2->unregister_memory(fake) == 0);  // now unpinned again
            delete t2;
        }
    }
    CHECK(photon::new_hip_vdma_target(nullptr, 100, 4096) == nullptr);  // size < unit
    CHECK(photon::new_hip_vdma_initiator("/photon_crc_vdma_absent", 0) == nullptr);

    delete target;
    printf("vdma local: %d failures\n", g_fail);
    return g_fail ? 1 : 0;
}

static int run_target(const char* name) {
    const size_t unit = 1 << 20, size = 8 << 20;
    photon::vDMATarget* target = photon::new_hip_vdma_target(name, size, unit);
    if (!target) {
        printf("FAIL target: %s\n", photon_crc_last_error());
        return 1;
    }
    photon::vDMABuffer* b[3];
    for (int k = 0; k < 3; ++k) {
        b[k] = target->alloc(unit);
        std::vector<uint8_t> h = pattern(k, unit);
        if (!b[k] || hipMemcpy(b[k]->address(), h.data(), unit, hipMemcpyHostToDevice) != hipSuccess) {
            printf("FAIL target fill\n");
            return 1;
        }
        printf("buffer %d %s %08x\n", k, hex(b[k]->id()).c_str(), crc32c(h.data(), unit));
    }
    printf("ready\n");
    fflush(stdout);
    std::string cmd;
    while (std::getline(std::cin, cmd)) {
        if (cmd == "check") {
            uint32_t c = 0;
            photon::vDMABuffer* one[1] = {b[2]};
            const int rc = photon::crc32c_vdma_batch(one, nullptr, 1, &c);
            printf("target-crc2 %d %08x\n", rc, c);
            fflush(stdout);
        } else if (cmd == "quit") {
            break;
        }
    }
    for (auto* x : b) target->dealloc(x);
    delete target;  // unlinks the published handle
    return 0;
}

static int run_initiator(const char* name, char** ids) {
    photon::vDMAInitiator* ini = photon::new_hip_vdma_initiator(name, 8 << 20);
    if (!ini) {
        printf("FAIL initiator: %s\n", photon_crc_last_error());
        return 1;
    }
    photon::vDMABuffer* b[3];
    for (int k = 0; k < 3; ++k) {
        b[k] = ini->map(unhex(ids[k]));
        CHECK(b[k] != nullptr);
        if (!b[k]) return 1;
        CHECK(b[k]->buf_size() == (1u << 20) && hex(b[k]->id()) == ids[k]);
    }
    CHECK(ini->map(unhex(ids[0])) == nullptr);  // mapped twice (shm.cpp:266-273)
    uint32_t crc[3];
    CHECK(photon::crc32c_vdma_batch(b, nullptr, 3, crc) == 0);
    for (int k = 0; k < 3; ++k) printf("initiator-crc %d %08x\n", k, crc[k]);
    // Overwrite buffer 2 from this process and hand it to the target.
    std::vector<uint8_t> h = pattern(99, 1 << 20);
    CHECK(hipMemcpy(b[2]->address(), h.data(), h.size(), hipMemcpyHostToDevice) == hipSuccess);
    CHECK(ini->write(b[2], h.size(), 0) == 0);
    CHECK(ini->write(b[2], 16, (off_t)h.size()) == -1);  // outside the buffer
    CHECK(ini->read(b[2], h.size(), 0) == 0);
    printf("initiator-wrote2 %08x\n", crc32c(h.data(), h.size()));
    for (auto* x : b) CHECK(ini->unmap(x) == 0);
    delete ini;
    printf("vdma initiator: %d failures\n", g_fail);
    return g_fail ? 1 : 0;
}

int main(int argc, char** argv) {
    if (photon_crc_device_count() <= 0) {
        fprintf(stderr, "no device: %s\n", photon_crc_last_error());
        return 2;
    }
    const std::string mode = argc > 1 ? argv[1] : "local";
    if (mode == "local") return local_checks();
    if (mode == "target" && argc > 2) return run_target(argv[2]);
    if (mode == "initiator" && argc > 5) return run_initiator(argv[2], argv + 3);
    fprintf(stderr, "usage: vdma_test local | target NAME | initiator NAME ID0 ID1 ID2\n");
    return 2;
}
