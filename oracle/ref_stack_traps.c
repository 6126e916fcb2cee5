/*
 * ref_stack_traps.c -- the mTCP stack functions that the reference objects
 * of ref_stack_harness.c reference but the checksum path never reaches
 * (TEST INFRASTRUCTURE ONLY).  No reference header is included: these are
 * link-time boundaries, not implementations.
 *
 *   StreamHTSearch   the first call ProcessTCPPacket makes after its checksum
 *                    prefix (tcp_in.c:1251): a longjmp back to the harness,
 *                    which records the frame as accepted.
 *   thread_printf    the TRACE_* logger (debug.h:241): output dropped.
 *   everything else  aborts: reaching it would mean the harness left the
 *                    checksum path.  (timer.c's list functions are the
 *                    reference's own, compiled in: SendTCPPacket calls them.)
 */
#include <setjmp.h>
#include <stdio.h>
#include <stdlib.h>

jmp_buf refs_accept_jb;
int refs_accept_armed;

void *StreamHTSearch(void *ht, const void *it)
{
	(void)ht; (void)it;
	if (!refs_accept_armed) {
		fprintf(stderr, "ref_stack: StreamHTSearch outside an RX frame\n");
		abort();
	}
	longjmp(refs_accept_jb, 1);
}

void thread_printf(void *mtcp, FILE *f, const char *fmt, ...)
{
	(void)mtcp; (void)f; (void)fmt;
}

#define TRAP(name) \
	void name(void) { fprintf(stderr, "ref_stack: trap %s reached\n", #name); abort(); }

TRAP(AddEpollEvent)
TRAP(CreateTCPStream)
TRAP(DestroyTCPStream)
TRAP(ListenerHTSearch)
TRAP(RBInit)
TRAP(RBPut)
TRAP(RBRemove)
TRAP(RaiseCloseEvent)
TRAP(RaiseErrorEvent)
TRAP(RaiseReadEvent)
TRAP(RaiseWriteEvent)
TRAP(SBRemove)
TRAP(StreamEnqueue)
