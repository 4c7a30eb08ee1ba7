// quarantine.c -- delayed free() for the reference app's benchmark run (TEST INFRASTRUCTURE ONLY).
//
// Linked into integration/_app/tyche_q only.  The executable defines free()
// (exported with -rdynamic), so every free() in the process -- the reference's
// objects and the shared libraries alike -- parks the block in a ring of
// kSlots entries and releases the oldest one through glibc's __libc_free.  The
// reference reads a Buffer after list__add_cow has destroyed it (clock_hand,
// list.c:714-722 vs 796, 1231-1234); with the block still parked the
// read sees the Buffer's last contents, as it did under jemalloc's layout.
// Also prints a backtrace on SIGSEGV/SIGABRT, so a crash in the run names its
// frame, and line-buffers stdout.
#include <dirent.h>
#include <execinfo.h>
#include <stdint.h>
#include <sys/syscall.h>
#include <pthread.h>
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <unistd.h>

#define kSlots 65536
void __libc_free(void *p);

static void *ring[kSlots];
static unsigned head;
static pthread_mutex_t mu = PTHREAD_MUTEX_INITIALIZER;

void free(void *p) {
    if (!p) return;
    pthread_mutex_lock(&mu);
    void *old = ring[head];
    ring[head] = p;
    head = (head + 1) % kSlots;
    pthread_mutex_unlock(&mu);
    if (old) __libc_free(old);
}

static void on_fault(int sig) {
    static const char msg[] = "\n*** fatal signal in the reference app; backtrace:\n";
    void *bt[64];
    (void)!write(2, msg, sizeof(msg) - 1);
    const int n = backtrace(bt, 64);
    backtrace_symbols_fd(bt, n, 2);
    signal(sig, SIG_DFL);
    raise(sig);
}

// TYCHE_APP_WATCHDOG=<seconds>: if the process is still alive then, every
// thread prints its backtrace (SIGUSR1 to each task) and the process exits
// with status 3 -- names the frames a hung run is waiting in.  A binary that
// defines tyche_app_report (batched_stats.c) has it called first: _exit runs
// no atexit handlers.
__attribute__((weak)) void tyche_app_report(void);
static void on_dump(int sig) {
    (void)sig;
    char hdr[64];
    const int k = snprintf(hdr, sizeof hdr, "\n--- thread %ld\n", (long)syscall(SYS_gettid));
    (void)!write(2, hdr, (size_t)k);
    void *bt[32];
    const int n = backtrace(bt, 32);
    backtrace_symbols_fd(bt, n, 2);
}
static void *watchdog(void *arg) {
    const unsigned secs = (unsigned)(uintptr_t)arg;
    sleep(secs);
    signal(SIGUSR1, on_dump);
    DIR *d = opendir("/proc/self/task");
    if (d) {
        struct dirent *e;
        const long self = (long)syscall(SYS_gettid);
        while ((e = readdir(d)) != NULL) {
            const long tid = atol(e->d_name);
            if (tid > 0 && tid != self) {
                syscall(SYS_tgkill, (long)getpid(), tid, SIGUSR1);
                usleep(2000);
            }
        }
        closedir(d);
    }
    usleep(200000);
    if (tyche_app_report) tyche_app_report();
    _exit(3);
    return NULL;
}

__attribute__((constructor)) static void install(void) {
    const char *wd = getenv("TYCHE_APP_WATCHDOG");
    if (wd && atoi(wd) > 0) {
        pthread_t t;
        pthread_create(&t, NULL, watchdog, (void *)(uintptr_t)atoi(wd));
        pthread_detach(t);
    }
    setvbuf(stdout, NULL, _IOLBF, 0);   // results survive a kill at shutdown (the reference can hang there)
    signal(SIGSEGV, on_fault);
    signal(SIGABRT, on_fault);
    signal(SIGBUS, on_fault);
}
