// Last words for a process that dies on a fatal signal (shmemx_set_fatal_note).
//
// The library's FATAL path aborts (runtime.cpp fatal(); the reference's
// trace.c:424-427 exits likewise), the HSA runtime aborts on a GPU memory
// fault, and torch.distributed.run sends SIGTERM to the surviving ranks when
// one rank dies.  A caller that has already computed a result it must not
// lose (bench.py's headline line, measured and verified before its optional
// extras run) registers that text here: on SIGABRT/SIGSEGV/SIGBUS/SIGFPE/
// SIGILL/SIGTERM the handler writes it to stdout with write(2) and leaves with
// _exit — both async-signal-safe, from whichever thread took the signal.  The
// exit status still says what happened: 128 + the signal number for a crash
// of this process (SIGABRT: a FATAL line or a GPU fault; SIGSEGV, SIGBUS,
// SIGFPE, SIGILL), the registered exit_code only for SIGTERM (the launcher
// stopping a healthy rank because another one died).  Registering NULL
// restores the previous dispositions.
//
// A note is one immutable block published by a single atomic pointer store,
// so a handler running on another thread sees either the old note or the new
// one, never a mix.  Replaced notes are not freed (a handler may still be
// reading one); callers register a handful per process.
#include <atomic>
#include <csignal>
#include <cstdlib>
#include <cstring>
#include <unistd.h>

#include "mirror.h"
#include "shmem_reduce_mi355x.h"

namespace {

constexpr int kSignals[] = {SIGABRT, SIGSEGV, SIGBUS, SIGFPE, SIGILL, SIGTERM};
constexpr int kNumSignals = sizeof kSignals / sizeof kSignals[0];

struct Note {
    const Note *older;   // notes are retired, never freed: kept reachable here
    int exit_code;
    size_t len;
    char text[1];
};

struct sigaction g_prev[kNumSignals];
bool g_installed = false;
std::atomic<const Note *> g_note{nullptr};
const Note *g_newest = nullptr;   // every note ever registered, newest first
std::atomic<int> g_fired{0};

void on_fatal(int sig, siginfo_t *si, void *) {
    // a fault of the mirrored heap's host view is not fatal: resolve it and
    // let the access run again (mirror.h)
    if (sig == SIGSEGV && si && shmx::mirror::handle_fault(si->si_addr)) return;
    const Note *n = g_note.load(std::memory_order_acquire);
    const int code = (n && sig == SIGTERM) ? n->exit_code : 128 + sig;
    if (g_fired.exchange(1)) _exit(code);     // a second signal while writing
    const char *p = n ? n->text : nullptr;
    size_t left = n ? n->len : 0;
    while (left > 0) {
        ssize_t w = write(STDOUT_FILENO, p, left);
        if (w <= 0) break;
        p += w;
        left -= static_cast<size_t>(w);
    }
    _exit(code);
}

}  // namespace

extern "C" int shmemx_set_fatal_note(const char *text, int exit_code) {
    if (text == nullptr) {
        if (g_installed) {
            for (int i = 0; i < kNumSignals; ++i) {
                // SIGSEGV: a mirrored heap created after the note was
                // installed chained its handler to ours; what we saved
                // predates it, so the view's handler goes back in front
                // (chaining to that saved disposition), not away
                if (kSignals[i] == SIGSEGV && shmx::mirror::active())
                    shmx::mirror::install_handler(&g_prev[i]);
                else
                    sigaction(kSignals[i], &g_prev[i], nullptr);
            }
            g_installed = false;
        }
        g_note.store(nullptr, std::memory_order_release);
        return SHMEMX_OK;
    }
    const size_t len = strlen(text);
    Note *n = static_cast<Note *>(malloc(sizeof(Note) + len));
    if (!n) return SHMEMX_ENOMEM;
    n->older = g_newest;
    g_newest = n;
    n->exit_code = exit_code;
    n->len = len;
    memcpy(n->text, text, len + 1);
    g_note.store(n, std::memory_order_release);
    if (!g_installed) {
        struct sigaction sa;
        memset(&sa, 0, sizeof sa);
        sa.sa_sigaction = on_fatal;
        sa.sa_flags = SA_SIGINFO | SA_NODEFER;
        sigfillset(&sa.sa_mask);
        for (int i = 0; i < kNumSignals; ++i) sigaction(kSignals[i], &sa, &g_prev[i]);
        g_installed = true;
    }
    return SHMEMX_OK;
}
