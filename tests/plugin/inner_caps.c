/*
 * inner_caps.c -- TEST ONLY.  Defines mTCP's module symbols the decorator
 * references weakly (dpdk_module_func, netmap_module_func), exported from the
 * executable (-rdynamic) as they would be from a linked mTCP, and prints the
 * caps gpucsum_set_inner picks for each inner module.  No GPU call is made.
 * -DWITH_IP_DEFRAG: the DPDK module of an IP_DEFRAG build (RX_ONCE).
 */
#include <stdio.h>

#include "../../include/mtcp_gpucsum.h"
#include "../../include/gpucsum_io_module.h"

io_module_func dpdk_module_func;
io_module_func netmap_module_func;
#ifdef WITH_IP_DEFRAG
/* what the integration patch adds to a dpdk_module.c built with IP_DEFRAG */
const int dpdk_module_ip_defrag = 1;
#endif
static io_module_func other_module;

int main(void)
{
	if (gpucsum_set_inner(&dpdk_module_func)) return 1;
	printf("dpdk %u\n", gpucsum_get_inner_caps());
	if (gpucsum_set_inner(&netmap_module_func)) return 1;
	printf("netmap %u\n", gpucsum_get_inner_caps());
	if (gpucsum_set_inner(&other_module)) return 1;
	printf("other %u\n", gpucsum_get_inner_caps());
	if (gpucsum_set_inner_caps(GPUCSUM_INNER_RX_CHAINED, 9000)) return 1;
	printf("set %u\n", gpucsum_get_inner_caps());
	return 0;
}
