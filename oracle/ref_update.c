/* Test infrastructure only (oracle/): exposes the reference's own
 * in_cksum_update -- the inline (or macro) of
 * /root/reference/sys/amd64/include/in_cksum.h:46-72 -- as an ordinary function,
 * so that tests can compare include/uinet_cksum.h's in_cksum_update with the
 * reference's output.  Compiled by oracle/Makefile with the reference's kernel
 * flags and include paths (the same environment as in_cksum.c, whose include
 * set this mirrors: in_cksum.c:40-49) and linked into _ref/libref_cksum.so. */
#include <sys/cdefs.h>
#include <sys/param.h>
#include <sys/mbuf.h>
#include <sys/systm.h>
#include <netinet/in_systm.h>
#include <netinet/in.h>
#include <netinet/ip.h>
#include <machine/in_cksum.h>

void ref_in_cksum_update(void *hdr);

void ref_in_cksum_update(void *hdr)
{
	struct ip *ip = hdr;
	in_cksum_update(ip);
}
