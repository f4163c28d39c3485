/* Minimal sampling profiler for host code (no perf in this image): LD_PRELOAD=sprof.so <program>.
 * SIGPROF every SPROF_US microseconds of process CPU time (default 500); the handler stores the
 * interrupted instruction pointer.  At exit the samples and /proc/self/maps go to
 * $SPROF_OUT (default /tmp/sprof.out); tools/sprof/report.py symbolizes them (addr2line -f -i).
 * SPROF_START_S=<s> drops the samples of the first seconds (wall time; the kernel delivers at most
 * one SIGPROF per tick, so sample counts are a poor clock).
 * Build: gcc -O2 -shared -fPIC tools/sprof/sprof.c -o /tmp/sprof.so */
#define _GNU_SOURCE
#include <signal.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/time.h>
#include <time.h>
#include <ucontext.h>

#define MAXS (1 << 24)
static unsigned long *samples;
static volatile long nsamples, nskip;
static long skip;   /* SPROF_SKIP: ignore the first samples (e.g. the opening of a run) */
static double start_after;   /* SPROF_START_S: ignore samples in the first seconds of wall time */
static double stop_after;    /* SPROF_STOP_S: ... and after this many seconds (0: never) */
static struct timespec t_init;
static double since_init(void) {
    struct timespec t;
    clock_gettime(CLOCK_MONOTONIC, &t);
    return (t.tv_sec - t_init.tv_sec) + 1e-9 * (t.tv_nsec - t_init.tv_nsec);
}

static void handler(int sig, siginfo_t *si, void *ctx) {
    (void)sig; (void)si;
    ucontext_t *uc = (ucontext_t *)ctx;
    if (__atomic_fetch_add(&nskip, 1, __ATOMIC_RELAXED) < skip) return;
    if (start_after > 0 || stop_after > 0) {
        const double t = since_init();
        if (t < start_after || (stop_after > 0 && t > stop_after)) return;
    }
    long i = __atomic_fetch_add(&nsamples, 1, __ATOMIC_RELAXED);
    if (i < MAXS) samples[i] = (unsigned long)uc->uc_mcontext.gregs[REG_RIP];
}

__attribute__((constructor)) static void sprof_init(void) {
    samples = (unsigned long *)malloc(sizeof(unsigned long) * MAXS);
    struct sigaction sa;
    memset(&sa, 0, sizeof(sa));
    sa.sa_sigaction = handler;
    sa.sa_flags = SA_SIGINFO | SA_RESTART;
    sigaction(SIGPROF, &sa, NULL);
    clock_gettime(CLOCK_MONOTONIC, &t_init);
    const char *st = getenv("SPROF_START_S");
    start_after = st ? atof(st) : 0;
    const char *sp = getenv("SPROF_STOP_S");
    stop_after = sp ? atof(sp) : 0;
    const char *sk = getenv("SPROF_SKIP");
    skip = sk ? atol(sk) : 0;
    const char *us = getenv("SPROF_US");
    long period = us ? atol(us) : 500;
    struct itimerval it;
    it.it_interval.tv_sec = period / 1000000;
    it.it_interval.tv_usec = period % 1000000;
    it.it_value = it.it_interval;
    setitimer(ITIMER_PROF, &it, NULL);
}

__attribute__((destructor)) static void sprof_fini(void) {
    struct itimerval it;
    memset(&it, 0, sizeof(it));
    setitimer(ITIMER_PROF, &it, NULL);
    const char *path = getenv("SPROF_OUT");
    FILE *f = fopen(path ? path : "/tmp/sprof.out", "w");
    if (!f) return;
    FILE *m = fopen("/proc/self/maps", "r");
    char line[4096];
    while (m && fgets(line, sizeof(line), m)) fprintf(f, "M %s", line);
    if (m) fclose(m);
    long n = nsamples < MAXS ? nsamples : MAXS;
    for (long i = 0; i < n; ++i) fprintf(f, "S %lx\n", samples[i]);
    fclose(f);
}
