/* Diagnostic: a SIGSEGV handler that prints the native backtrace (with dladdr symbols) to
 * stderr, loaded by ctypes (tools/capture_probe.py with LGCN_SEGV_TRACE=1) to locate a host
 * crash inside the HIP runtime.  gcc -O1 -g -shared -fPIC -o tools/libsegv_trace.so tools/segv_trace.c -ldl */
#define _GNU_SOURCE
#include <dlfcn.h>
#include <execinfo.h>
#include <signal.h>
#include <stdio.h>
#include <string.h>
#include <unistd.h>

static void handler(int sig, siginfo_t* si, void* ctx) {
    (void)ctx;
    void* bt[64];
    int n = backtrace(bt, 64);
    fprintf(stderr, "=== signal %d at address %p, %d frames\n", sig, si->si_addr, n);
    for (int i = 0; i < n; ++i) {
        Dl_info info;
        if (dladdr(bt[i], &info) && info.dli_fname) {
            fprintf(stderr, "  #%d %p %s(%s+0x%lx)\n", i, bt[i], info.dli_fname,
                    info.dli_sname ? info.dli_sname : "?",
                    (unsigned long)((char*)bt[i] - (char*)(info.dli_saddr ? info.dli_saddr : info.dli_fbase)));
        } else {
            fprintf(stderr, "  #%d %p\n", i, bt[i]);
        }
    }
    fflush(stderr);
    signal(sig, SIG_DFL);
    raise(sig);
}

void segv_install(void);
__attribute__((constructor)) static void install(void) { segv_install(); }

void segv_install(void) {
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = handler;
    sa.sa_flags = SA_SIGINFO | SA_RESETHAND;
    sigaction(SIGSEGV, &sa, NULL);
    sigaction(SIGBUS, &sa, NULL);
}
