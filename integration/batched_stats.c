/* batched_stats.c -- linked into _app/tyche_batched only (TEST INFRASTRUCTURE):
 * at exit (and from quarantine.c's watchdog before its _exit), prints the engine's restore-queue counters (launches and buffers
 * served, tyche_restore_queue_stats) and the sweep batches (tyche_buffers_compress
 * calls and buffers) so the C1 batched test can see that the reference's own
 * callers drove batched GPU work. */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <unistd.h>

void tyche_restore_queue_stats(uint64_t *batches, uint64_t *buffers);

/* formatted on the stack and written with write(2), not stdio: the watchdog calls this while other
 * threads are stopped at arbitrary points, possibly holding stderr's FILE lock */
void tyche_app_report(void) {
    uint64_t batches = 0, buffers = 0;
    tyche_restore_queue_stats(&batches, &buffers);
    char line[96];
    const int k = snprintf(line, sizeof line, "tyche-restore-queue: batches %llu buffers %llu\n",
                           (unsigned long long)batches, (unsigned long long)buffers);
    if (k > 0) (void)!write(2, line, (size_t)k < sizeof line ? (size_t)k : sizeof line - 1);
}

__attribute__((constructor)) static void register_report(void) { atexit(tyche_app_report); }
