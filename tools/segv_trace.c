/* segv_trace.c -- diagnostic: a SIGSEGV/SIGBUS handler that prints the native backtrace
 * (backtrace_symbols_fd: "lib.so(+offset)", symbolize offline with llvm-symbolizer against the
 * same build) and then hands the signal to the previous handler (Python's faulthandler prints the
 * Python frames).  Loaded by ctypes from a test that needs it; never part of the product.
 * build: gcc -O1 -g -shared -fPIC -o tools/libsegv_trace.so tools/segv_trace.c */
#define _GNU_SOURCE
#include <execinfo.h>
#include <signal.h>
#include <string.h>
#include <unistd.h>

static struct sigaction prev_segv, prev_bus;

static void on_fault(int sig, siginfo_t *si, void *uc) {
    void *frames[64];
    const char msg[] = "\n=== native backtrace (segv_trace) ===\n";
    if (write(2, msg, sizeof msg - 1) < 0) { }
    int n = backtrace(frames, 64);
    backtrace_symbols_fd(frames, n, 2);
    struct sigaction *p = sig == SIGSEGV ? &prev_segv : &prev_bus;
    if (p->sa_flags & SA_SIGINFO) {
        if (p->sa_sigaction) { p->sa_sigaction(sig, si, uc); return; }
    } else if (p->sa_handler != SIG_DFL && p->sa_handler != SIG_IGN) {
        p->sa_handler(sig);
        return;
    }
    signal(sig, SIG_DFL);
    raise(sig);
}

static char altstack[1 << 16];

/* (Re)install the handler now, on an alternate stack for the calling thread: call it right before
 * the code under suspicion (a later faulthandler.enable() would otherwise sit in front of it). */
void segv_trace_install(void) {
    stack_t ss;
    ss.ss_sp = altstack;
    ss.ss_size = sizeof altstack;
    ss.ss_flags = 0;
    sigaltstack(&ss, NULL);
    struct sigaction sa;
    memset(&sa, 0, sizeof sa);
    sa.sa_sigaction = on_fault;
    sa.sa_flags = SA_SIGINFO | SA_ONSTACK;
    sigemptyset(&sa.sa_mask);
    struct sigaction old;
    sigaction(SIGSEGV, &sa, &old);
    if (!((old.sa_flags & SA_SIGINFO) && old.sa_sigaction == on_fault)) prev_segv = old;   /* never chain to itself */
    sigaction(SIGBUS, &sa, &old);
    if (!((old.sa_flags & SA_SIGINFO) && old.sa_sigaction == on_fault)) prev_bus = old;
}

__attribute__((constructor)) static void install(void) { segv_trace_install(); }
