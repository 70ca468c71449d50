// Host test of the mirrored heap's core (openshmem-async_amd/csrc/mirror.cpp):
// block states, page protection and the SIGSEGV path, with a memcpy backend
// standing in for HIP (the "device segment" is a plain host buffer).  Random
// sequences of host stores / loads and collective-style flush + device
// writes are checked against a model: after every step the host view reads
// what the model says, flush pushes exactly the blocks the host stored to,
// and nothing else crosses the "PCIe" backend.
#include <sys/wait.h>
#include <unistd.h>

#include <atomic>
#include <cerrno>
#include <chrono>
#include <thread>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <vector>

#include "mirror.h"
#include "shmem_reduce_mi355x.h"   // shmemx_set_fatal_note (fatal_note.cpp)

namespace M = shmx::mirror;

static int fails = 0;
#define CHECK(c)                                                        \
    do {                                                                \
        if (!(c)) {                                                     \
            std::printf("FAIL %s:%d %s\n", __FILE__, __LINE__, #c);    \
            ++fails;                                                    \
        }                                                               \
    } while (0)

static std::vector<unsigned char> g_dev;   // the "device segment"
static volatile size_t g_h2d = 0, g_d2h = 0;   // bytes moved

// a hook the flush race test runs inside to_device, between the view's
// protection change and the copy (another thread's store lands there)
static void (*g_in_to_device)() = nullptr;

// the backend works on the view's always-writable alias
static void to_device(uint64_t off, size_t bytes, void *) {
    if (g_in_to_device) g_in_to_device();
    std::memcpy(g_dev.data() + off, M::alias_base() + off, bytes);
    g_h2d += bytes;
}
static void to_host(uint64_t off, size_t bytes, void *) {
    std::memcpy(M::alias_base() + off, g_dev.data() + off, bytes);
    g_d2h += bytes;
}
static void drain(void *) {}

int main(int argc, char **argv) {
    const int iters = argc > 1 ? std::atoi(argv[1]) : 2000;
    const size_t nblocks = 96, bytes = nblocks * M::kBlock;
    g_dev.assign(bytes, 0);
    CHECK(M::create(bytes, M::Backend{to_device, to_host, drain, nullptr}));
    // volatile: the fault handler changes the backend's counters and the
    // view's protection behind the compiler's back
    volatile unsigned char *h = reinterpret_cast<volatile unsigned char *>(M::host_base());
    CHECK(M::view_bytes() == bytes);
    // model: the value every byte must read as on the host (the truth)
    std::vector<unsigned char> truth(bytes, 0);

    // fresh view: zeros, CLEAN, loads never fault
    for (size_t i = 0; i < bytes; i += 4093) CHECK(h[i] == 0);
    CHECK(M::stats(false).write_faults == 0 && M::stats(false).read_faults == 0);

    // a store faults once and marks its block HOST_NEWER
    h[5] = 7;
    truth[5] = 7;
    CHECK(M::state_of(5) == M::HOST_NEWER);
    CHECK(M::stats(false).write_faults == 1);
    // a flush of a range that overlaps it pushes exactly that block
    CHECK(M::flush(0, 16) == 1);
    CHECK(g_h2d == M::kBlock && g_dev[5] == 7);
    CHECK(M::state_of(5) == M::CLEAN);
    CHECK(M::flush(0, bytes) == 0);   // nothing dirty any more

    // a sequential writer gets doubling runs: far fewer faults than blocks
    M::stats(true);
    for (size_t i = 0; i < 40 * M::kBlock; ++i) {
        h[8 * M::kBlock + i] = (unsigned char)(i * 13);
        truth[8 * M::kBlock + i] = (unsigned char)(i * 13);
    }
    const auto ws = M::stats(false).write_faults;
    CHECK(ws >= 2 && ws <= 8);
    std::printf("sequential 40 blocks: %llu write faults\n", (unsigned long long)ws);

    // a "collective" writes blocks 10..19 on the device: flush first, then
    // the host view of them faults and reads the device bytes
    g_h2d = 0;
    M::flush(10 * M::kBlock, 10 * M::kBlock);
    for (size_t i = 10 * M::kBlock; i < 20 * M::kBlock; ++i) {
        g_dev[i] = (unsigned char)(i * 7 + 1);
        truth[i] = g_dev[i];
    }
    CHECK(M::device_wrote(10 * M::kBlock, 10 * M::kBlock) == 10);
    CHECK(M::state_of(10 * M::kBlock) == M::DEVICE_NEWER);
    g_d2h = 0;
    CHECK(h[15 * M::kBlock + 3] == truth[15 * M::kBlock + 3]);   // a load faults, fetches a run
    CHECK(g_d2h == M::kBlock);                                   // block 15 alone (a first fault)
    CHECK(M::state_of(15 * M::kBlock) == M::CLEAN && M::state_of(16 * M::kBlock) == M::DEVICE_NEWER);
    CHECK(h[16 * M::kBlock] == truth[16 * M::kBlock] && g_d2h == 3 * M::kBlock);   // sequential: 2 more
    h[11 * M::kBlock] = 99;                                       // a store: fetch, then dirty
    truth[11 * M::kBlock] = 99;
    CHECK(M::state_of(11 * M::kBlock) == M::HOST_NEWER);
    CHECK(h[11 * M::kBlock + 1] == truth[11 * M::kBlock + 1]);

    // system calls do not take the page fault: on a block the library has
    // not opened they fail with EFAULT, and acquire() opens the range
    {
        int fds[2];
        CHECK(pipe(fds) == 0);
        M::flush(40 * M::kBlock, 2 * M::kBlock);
        for (size_t i = 40 * M::kBlock; i < 42 * M::kBlock; ++i) {
            g_dev[i] = (unsigned char)(i * 5 + 3);
            truth[i] = g_dev[i];
        }
        M::device_wrote(40 * M::kBlock, 2 * M::kBlock);
        const char *v = M::host_base();
        errno = 0;
        CHECK(write(fds[1], v + 40 * M::kBlock + 100, 1000) == -1 && errno == EFAULT);
        CHECK(M::acquire(40 * M::kBlock + 100, 1000, false) == 1);   // one block back
        CHECK(M::state_of(40 * M::kBlock) == M::CLEAN && M::state_of(41 * M::kBlock) == M::DEVICE_NEWER);
        CHECK(write(fds[1], v + 40 * M::kBlock + 100, 1000) == 1000);
        unsigned char buf[1000];
        CHECK(read(fds[0], buf, 1000) == 1000);
        CHECK(std::memcmp(buf, truth.data() + 40 * M::kBlock + 100, 1000) == 0);
        // read(2) into a CLEAN (read-only) block: EFAULT until acquired for writing
        std::memset(buf, 0x5A, sizeof buf);
        CHECK(write(fds[1], buf, 1000) == 1000);
        errno = 0;
        CHECK(read(fds[0], const_cast<char *>(v) + 40 * M::kBlock + 7, 1000) == -1 && errno == EFAULT);
        CHECK(M::acquire(40 * M::kBlock + 7, 1000, true) == 0);
        CHECK(M::state_of(40 * M::kBlock) == M::HOST_NEWER);
        CHECK(read(fds[0], const_cast<char *>(v) + 40 * M::kBlock + 7, 1000) == 1000);
        std::memset(truth.data() + 40 * M::kBlock + 7, 0x5A, 1000);
        g_h2d = 0;
        CHECK(M::flush(40 * M::kBlock, 1) == 1 && g_dev[40 * M::kBlock + 7] == 0x5A);
        // acquire for writing across a DEVICE_NEWER block fetches it first
        CHECK(M::acquire(41 * M::kBlock, 10, true) == 1 && M::state_of(41 * M::kBlock) == M::HOST_NEWER);
        CHECK(h[41 * M::kBlock + 5] == truth[41 * M::kBlock + 5]);
        close(fds[0]);
        close(fds[1]);
    }

    // Two threads.  (1) A collective writes a 64-byte target at the start of
    // block 50 while another thread stores to a neighbouring object in the
    // same block: the store must wait for the write in flight, then land on
    // top of the collective's result — neither is lost.
    {
        const size_t base = 50 * M::kBlock;
        M::stats(true);
        CHECK(M::begin_device_write(base, 64) == 1);
        CHECK(M::state_of(base) == M::DEVICE_NEWER);
        std::atomic<int> stored{0};
        std::thread other([&] {
            h[base + 100] = 42;              // faults, waits for end_device_write
            stored.store(1);
        });
        std::this_thread::sleep_for(std::chrono::milliseconds(100));
        CHECK(stored.load() == 0);           // still waiting: the write is in flight
        for (size_t i = 0; i < 64; ++i) {    // the collective's result, "enqueued"
            g_dev[base + i] = (unsigned char)(200 + i);
            truth[base + i] = g_dev[base + i];
        }
        M::end_device_write(base, 64);
        other.join();
        truth[base + 100] = 42;
        CHECK(stored.load() == 1);
        for (size_t i = 0; i < 128; ++i) CHECK(h[base + i] == truth[base + i]);
        CHECK(M::state_of(base) == M::HOST_NEWER && M::stats(false).fault_waits >= 1);
        CHECK(M::flush(base, 1) == 1 && g_dev[base + 100] == 42 && g_dev[base + 3] == 203);
    }
    // (1b) A write in flight on one block does not hold up a fault on another
    // (ADVICE r03): block 52 is DEVICE_NEWER from an earlier collective while
    // a new one is being enqueued on block 51; a load from block 52 fetches
    // at once.
    {
        const size_t w = 51 * M::kBlock, other_blk = 52 * M::kBlock;
        M::flush(w, 2 * M::kBlock);
        for (size_t i = other_blk; i < other_blk + 16; ++i) {
            g_dev[i] = (unsigned char)(i * 7);
            truth[i] = g_dev[i];
        }
        M::device_wrote(other_blk, 16);
        CHECK(M::begin_device_write(w, 8) == 1);
        std::atomic<int> loaded{0};
        std::thread reader([&] {
            loaded.store(h[other_blk + 3] == truth[other_blk + 3] ? 1 : 2);
        });
        for (int k = 0; k < 200 && !loaded.load(); ++k) std::this_thread::sleep_for(std::chrono::milliseconds(5));
        CHECK(loaded.load() == 1);           // not waiting for block 51's write
        for (size_t i = 0; i < 8; ++i) {
            g_dev[w + i] = (unsigned char)(90 + i);
            truth[w + i] = g_dev[w + i];
        }
        M::end_device_write(w, 8);
        reader.join();
        CHECK(h[w + 2] == truth[w + 2]);
    }
    // (1b') A sequential reader's fetch run stops at a block with a write in
    // flight: block 59 is being written while 57 and 58 are read in turn (the
    // second fault would fetch a run of two), so 59 stays DEVICE_NEWER until
    // its write ends, and then reads the collective's bytes.
    {
        const size_t b57 = 57 * M::kBlock, b59 = 59 * M::kBlock;
        M::flush(b57, 3 * M::kBlock);
        for (size_t i = b57; i < b57 + 3 * M::kBlock; i += 4096) {
            g_dev[i] = (unsigned char)(i / 4096 + 11);
            truth[i] = g_dev[i];
        }
        M::device_wrote(b57, 2 * M::kBlock);
        CHECK(M::begin_device_write(b59, 16) == 1);
        CHECK(h[b57] == truth[b57]);                        // first fault: block 57 alone
        CHECK(h[b57 + M::kBlock] == truth[b57 + M::kBlock]);  // sequential: would take 58 and 59
        CHECK(M::state_of(b59) == M::DEVICE_NEWER);          // 59 is not fetched while being written
        g_dev[b59] = 0x3C;
        truth[b59] = 0x3C;
        M::end_device_write(b59, 16);
        CHECK(h[b59] == 0x3C);
    }
    // (1c) settle(): a blocking call's small result comes back into the view
    // before the call returns.  A write on CLEAN blocks ("fresh") copies only
    // its own bytes back and leaves the blocks CLEAN (no fault afterwards, a
    // system call can read them); a write on a block that was already
    // DEVICE_NEWER fetches the whole block; a write still in flight on the
    // block makes settle() leave it alone.
    {
        const size_t b = 54 * M::kBlock + 100;
        M::flush(54 * M::kBlock, 3 * M::kBlock);
        bool fresh = false;
        CHECK(M::begin_device_write(b, 40, &fresh) == 1 && fresh);
        for (size_t i = 0; i < 40; ++i) {
            g_dev[b + i] = (unsigned char)(17 + i);
            truth[b + i] = g_dev[b + i];
        }
        M::end_device_write(b, 40);
        const size_t d2h0 = g_d2h;
        const auto rf0 = M::stats(false).read_faults;
        CHECK(M::settle(b, 40, fresh) == 40 && g_d2h - d2h0 == 40);
        CHECK(M::state_of(b) == M::CLEAN);
        for (size_t i = 54 * M::kBlock; i < 55 * M::kBlock; i += 7) CHECK(h[i] == truth[i]);
        CHECK(M::stats(false).read_faults == rf0);      // readable without a fault
        int fds[2];
        CHECK(pipe(fds) == 0);                          // and by a system call
        CHECK(write(fds[1], const_cast<unsigned char *>(h + b), 40) == 40);
        unsigned char got[40];
        CHECK(read(fds[0], got, 40) == 40 && std::memcmp(got, truth.data() + b, 40) == 0);
        close(fds[0]);
        close(fds[1]);
        // block 55 was DEVICE_NEWER already: not fresh, fetched whole
        const size_t c = 55 * M::kBlock;
        for (size_t i = c; i < c + M::kBlock; ++i) {
            g_dev[i] = (unsigned char)(i * 5);
            truth[i] = g_dev[i];
        }
        M::device_wrote(c, M::kBlock);
        CHECK(M::begin_device_write(c + 8, 8, &fresh) == 0 && !fresh);
        M::end_device_write(c + 8, 8);
        CHECK(M::settle(c + 8, 8, fresh) == M::kBlock && M::state_of(c) == M::CLEAN);
        CHECK(h[c + 1000] == truth[c + 1000]);
        // another write in flight on block 56: settle leaves it DEVICE_NEWER
        const size_t d = 56 * M::kBlock;
        CHECK(M::begin_device_write(d, 8, &fresh) == 1 && fresh);
        CHECK(M::begin_device_write(d + 64, 8) == 0);
        for (size_t i = 0; i < 72; ++i) {
            g_dev[d + i] = (unsigned char)(3 * i + 1);
            truth[d + i] = g_dev[d + i];
        }
        M::end_device_write(d, 8);
        CHECK(M::settle(d, 8, fresh) == 0 && M::state_of(d) == M::DEVICE_NEWER);
        M::end_device_write(d + 64, 8);
        CHECK(h[d + 65] == truth[d + 65] && M::state_of(d) == M::CLEAN);   // the fault path
        // the call's own stream already stored the result into the alias
        // (settle with `copied`): nothing more moves, the block is CLEAN
        const size_t e = 53 * M::kBlock + 40;
        M::flush(53 * M::kBlock, M::kBlock);
        CHECK(M::begin_device_write(e, 8, &fresh) == 1 && fresh);
        for (size_t i = 0; i < 8; ++i) {
            g_dev[e + i] = (unsigned char)(0xE0 + i);
            M::alias_base()[e + i] = (char)(0xE0 + i);     // the in-stream copy
            truth[e + i] = g_dev[e + i];
        }
        M::end_device_write(e, 8);
        const size_t d2h1 = g_d2h;
        const auto rf1 = M::stats(false).read_faults;
        CHECK(M::settle(e, 8, fresh, true) == 0 && g_d2h == d2h1 && M::state_of(e) == M::CLEAN);
        CHECK(h[e + 3] == truth[e + 3] && M::stats(false).read_faults == rf1);
    }
    // (1d) the light path of a blocking call on small operands: flush_bytes
    // sends only the operand's bytes of a HOST_NEWER block and leaves it
    // HOST_NEWER (writable: no fault on the next store); begin_light_write
    // keeps CLEAN / HOST_NEWER blocks as they are, refuses a block with a
    // write in flight or DEVICE_NEWER; end_light_write copies the result back
    // unless the call's stream did, and counts the blocks settled.
    {
        const size_t b = 62 * M::kBlock;
        h[b + 10] = 0x11;                      // HOST_NEWER (a write fault)
        h[b + 5000] = 0x22;
        truth[b + 10] = 0x11;
        truth[b + 5000] = 0x22;
        CHECK(M::state_of(b) == M::HOST_NEWER);
        M::flush(b + M::kBlock, M::kBlock);    // block 63 CLEAN (a write fault may open a run)
        const size_t h2d0 = g_h2d;
        const auto fl0 = M::stats(false).blocks_flushed;
        CHECK(M::flush_bytes(b + 8, 8) == 1 && g_h2d - h2d0 == 8 && g_dev[b + 10] == 0x11);
        CHECK(g_dev[b + 5000] != 0x22);        // the rest of the block stayed on the host
        CHECK(M::state_of(b) == M::HOST_NEWER && M::stats(false).blocks_flushed == fl0 + 1);
        const auto wf0 = M::stats(false).write_faults;
        h[b + 11] = 0x33;                      // still writable: no fault
        truth[b + 11] = 0x33;
        CHECK(M::stats(false).write_faults == wf0);
        CHECK(M::flush_bytes(b + M::kBlock, 8) == 0);   // block 63 is CLEAN: nothing moves
        // a light write on the HOST_NEWER block, the result also stored into
        // the alias by the call's stream: nothing changes state
        CHECK(M::begin_light_write(b + 64, 8));
        CHECK(M::state_of(b) == M::HOST_NEWER);
        CHECK(!M::begin_light_write(b + 128, 8));       // a write is in flight on block 62
        bool fresh = true;
        CHECK(M::begin_device_write(b + 2 * M::kBlock, 8, &fresh) == 1);   // block 64: in flight
        CHECK(!M::begin_light_write(b + 2 * M::kBlock + 64, 8));
        for (size_t i = 0; i < 8; ++i) {
            g_dev[b + 2 * M::kBlock + i] = (unsigned char)(0x70 + i);
            truth[b + 2 * M::kBlock + i] = g_dev[b + 2 * M::kBlock + i];
        }
        M::end_device_write(b + 2 * M::kBlock, 8);
        for (size_t i = 0; i < 8; ++i) {
            g_dev[b + 64 + i] = (unsigned char)(0xA0 + i);
            M::alias_base()[b + 64 + i] = (char)(0xA0 + i);
            truth[b + 64 + i] = g_dev[b + 64 + i];
        }
        const size_t d2h0 = g_d2h;
        const auto se0 = M::stats(false).blocks_settled;
        CHECK(M::end_light_write(b + 64, 8, true) == 0 && g_d2h == d2h0);
        CHECK(M::stats(false).blocks_settled == se0 + 1);
        CHECK(h[b + 67] == truth[b + 67] && M::state_of(b) == M::HOST_NEWER);
        // flushed whole later: HBM then holds the host's bytes and the result
        CHECK(M::flush(b, 1) == 1 && g_dev[b + 5000] == 0x22 && g_dev[b + 11] == 0x33 && g_dev[b + 64] == 0xA0);
        // on a CLEAN block without the stream's copy: end_light_write copies
        // the result's bytes back, and the block stays CLEAN and readable
        const size_t c = b + M::kBlock;
        CHECK(M::state_of(c) == M::CLEAN && M::begin_light_write(c + 16, 16));
        for (size_t i = 0; i < 16; ++i) {
            g_dev[c + 16 + i] = (unsigned char)(0x50 + i);
            truth[c + 16 + i] = g_dev[c + 16 + i];
        }
        const size_t d2h1 = g_d2h;
        const auto rf0 = M::stats(false).read_faults;
        CHECK(M::end_light_write(c + 16, 16, false) == 16 && g_d2h - d2h1 == 16);
        CHECK(M::state_of(c) == M::CLEAN && h[c + 20] == truth[c + 20] && M::stats(false).read_faults == rf0);
        // a DEVICE_NEWER block refuses the light path, and is left as it was
        M::device_wrote(c, M::kBlock);
        CHECK(!M::begin_light_write(c + 16, 8) && M::state_of(c) == M::DEVICE_NEWER);
        CHECK(h[c + 20] == truth[c + 20] && M::state_of(c) == M::CLEAN);   // fetched by the fault
    }
    // (2) A store another thread makes while a flush copies its block (after
    // the protection change, before the copy) is not lost: it faults, waits,
    // and leaves the block HOST_NEWER for the next flush.
    {
        const size_t base = 60 * M::kBlock;
        h[base] = 1;                          // HOST_NEWER
        truth[base] = 1;
        static std::atomic<int> phase{0};
        static volatile unsigned char *hv;
        static size_t racing;
        phase = 0;
        hv = h;
        racing = base + 777;
        std::thread other([] {
            while (phase.load() != 1) std::this_thread::yield();
            hv[racing] = 77;                  // faults (read-only now), waits for the lock
            phase.store(3);
        });
        g_in_to_device = [] {
            phase.store(1);
            std::this_thread::sleep_for(std::chrono::milliseconds(50));
            if (phase.load() == 3) ++fails;   // the racing store did not fault
        };
        CHECK(M::flush(base, 1) == 1);
        g_in_to_device = nullptr;
        other.join();
        truth[racing] = 77;
        CHECK(phase.load() == 3 && M::state_of(base) == M::HOST_NEWER);
        CHECK(M::flush(base, 1) == 1 && g_dev[racing] == 77 && g_dev[base] == 1);
    }

    // (3) A forked child has no fault service thread: its fault on a
    // device-newer block copies in place instead of waiting forever.
    {
        const size_t base = 70 * M::kBlock;
        M::flush(base, M::kBlock);
        for (size_t i = base; i < base + M::kBlock; ++i) {
            g_dev[i] = (unsigned char)(i * 3 + 1);
            truth[i] = g_dev[i];
        }
        M::device_wrote(base, M::kBlock);
        const pid_t pid = fork();
        if (pid == 0) {
            alarm(10);   // a hang fails the check instead of the suite
            const bool ok = h[base + 5] == truth[base + 5] && M::state_of(base) == M::CLEAN;
            _exit(ok ? 0 : 3);
        }
        int status = 0;
        CHECK(pid > 0 && waitpid(pid, &status, 0) == pid);
        CHECK(WIFEXITED(status) && WEXITSTATUS(status) == 0);
    }

    // random interleavings against the model
    std::mt19937_64 rng(12345);
    for (int it = 0; it < iters; ++it) {
        const int what = (int)(rng() % 5);
        const size_t off = rng() % bytes;
        const size_t len = 1 + rng() % (3 * M::kBlock);
        const size_t n = off + len > bytes ? bytes - off : len;
        if (what == 0) {            // host stores
            for (size_t i = off; i < off + n; i += 1 + rng() % 997) {
                const unsigned char v = (unsigned char)rng();
                h[i] = v;
                truth[i] = v;
            }
        } else if (what == 1) {     // host loads
            for (size_t i = off; i < off + n; i += 1 + rng() % 991) CHECK(h[i] == truth[i]);
        } else if (what == 2) {     // a collective reads the range on the device
            M::flush(off, n);
            for (size_t i = off; i < off + n; i += 1 + rng() % 983) CHECK(g_dev[i] == truth[i]);
        } else if (what == 4) {     // a blocking call on small operands (the light path)
            const size_t m = 1 + rng() % 4096;
            const size_t so = rng() % (bytes - m), to = rng() % (bytes - m);
            M::flush_bytes(so, m);
            for (size_t i = so; i < so + m; i += 1 + rng() % 97) CHECK(g_dev[i] == truth[i]);
            if (M::begin_light_write(to, m)) {
                const bool copied = rng() % 2;
                for (size_t i = to; i < to + m; ++i) {
                    g_dev[i] = (unsigned char)(i * 7 + it);
                    if (copied) M::alias_base()[i] = (char)g_dev[i];   // the call's stream
                    truth[i] = g_dev[i];
                }
                M::end_light_write(to, m, copied);
            } else {                // a block is DEVICE_NEWER: the ordinary marking
                M::begin_device_write(to, m);
                for (size_t i = to; i < to + m; ++i) {
                    g_dev[i] = (unsigned char)(i * 7 + it);
                    truth[i] = g_dev[i];
                }
                M::end_device_write(to, m);
            }
        } else {                    // a collective writes the range on the device
            M::flush(off, n);
            // the device holds the whole blocks' truth after the flush
            const size_t b0 = off / M::kBlock * M::kBlock;
            const size_t b1 = (off + n + M::kBlock - 1) / M::kBlock * M::kBlock;
            for (size_t i = b0; i < b1 && i < bytes; i += 1 + rng() % 977)
                CHECK(M::state_of(i) != M::HOST_NEWER && (M::state_of(i) == M::DEVICE_NEWER || g_dev[i] == truth[i]));
            for (size_t i = off; i < off + n; ++i) {
                g_dev[i] = (unsigned char)(i ^ it);
                truth[i] = g_dev[i];
            }
            M::device_wrote(off, n);
        }
        if (fails > 20) break;
    }
    // everything back on the host, and equal to the model
    M::fetch_all();
    CHECK(std::memcmp(const_cast<unsigned char *>(h), truth.data(), bytes) == 0);
    const auto st = M::stats(false);
    std::printf("stats: %llu write faults, %llu read faults, %llu flushed, %llu fetched blocks\n",
                (unsigned long long)st.write_faults, (unsigned long long)st.read_faults,
                (unsigned long long)st.blocks_flushed, (unsigned long long)st.blocks_fetched);
    M::destroy();

    // The fatal-note handler installed BEFORE the view exists, then removed:
    // what it saved predates the view's handler, and removing it must put
    // the view's handler back in front, not uninstall it (the next host
    // store to a CLEAN block would kill the process).
    CHECK(shmemx_set_fatal_note("last words\n", 3) == SHMEMX_OK);
    g_dev.assign(bytes, 0);
    CHECK(M::create(bytes, M::Backend{to_device, to_host, drain, nullptr}));
    CHECK(shmemx_set_fatal_note(nullptr, 0) == SHMEMX_OK);
    volatile unsigned char *h2 = reinterpret_cast<volatile unsigned char *>(M::host_base());
    h2[3 * M::kBlock + 9] = 5;                        // faults into the view's handler
    CHECK(M::state_of(3 * M::kBlock) == M::HOST_NEWER && h2[3 * M::kBlock + 9] == 5);
    M::destroy();
    if (fails) {
        std::printf("%d failures\n", fails);
        return 1;
    }
    std::printf("ok %d\n", iters);
    return 0;
}
