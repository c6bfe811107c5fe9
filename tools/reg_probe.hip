/*
 * reg_probe.hip -- diagnostic, not product code: what the HIP/ROCr runtime
 * records for a hipHostRegister'ed range when the same start address is
 * registered again after an unregister, with a larger size (the sequence
 * before every registered-memory fault of rounds 2-4).
 *
 * Only host-side queries (hsa_amd_pointer_info) follow the second
 * registration: nothing on the GPU ever touches a range whose lock is in
 * doubt.  The first registration is used by a DMA (a legal access) in some
 * variants, to see whether use changes what outlives the unregister.
 *
 *   tools/reg_probe            all variants, one line each
 */
#include <hip/hip_runtime.h>
#include <hsa/hsa_ext_amd.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/mman.h>

static void info(const char *tag, const void *p)
{
	hsa_amd_pointer_info_t in;
	memset(&in, 0, sizeof in);
	in.size = sizeof in;
	const hsa_status_t s = hsa_amd_pointer_info(p, &in, nullptr, nullptr, nullptr);
	hipPointerAttribute_t pa;
	memset(&pa, 0, sizeof pa);
	const hipError_t he = hipPointerGetAttributes(&pa, p);
	(void)hipGetLastError();
	printf("  %-28s ptr=%p rocr: status=%d type=%d host=%p agent=%p size=%zu registered=%d | "
	       "hip: %s type=%d dev=%p host=%p flags=%#x\n", tag, p,
	       (int)s, (int)in.type, in.hostBaseAddress, in.agentBaseAddress, in.sizeInBytes,
	       (int)in.registered, hipGetErrorName(he), (int)pa.type, pa.devicePointer,
	       pa.hostPointer, pa.allocationFlags);
}

#define CK(x)                                                                     \
	do {                                                                      \
		hipError_t e_ = (x);                                              \
		if (e_ != hipSuccess)                                             \
			printf("  %s -> %s\n", #x, hipGetErrorName(e_));          \
	} while (0)

/* small then large registration at one start address */
static void variant(const char *name, uint8_t *p, size_t small, size_t large, bool dma_first,
		    void *dbuf)
{
	printf("%s\n", name);
	info("before", p);
	CK(hipHostRegister(p, small, hipHostRegisterMapped));
	info("after register small", p);
	if (dma_first) {
		CK(hipMemcpy(dbuf, p, small, hipMemcpyHostToDevice));
		CK(hipDeviceSynchronize());
	}
	CK(hipHostUnregister(p));
	info("after unregister small", p);
	CK(hipHostRegister(p, large, hipHostRegisterMapped));
	info("after register large", p);
	info("  ... at its last byte", p + large - 1);
	CK(hipHostUnregister(p));
	info("after unregister large", p);
}

int main()
{
	int n = 0;
	if (hipGetDeviceCount(&n) != hipSuccess || n == 0) {
		printf("reg_probe: no GPU\n");
		return 77;
	}
	CK(hipSetDevice(0));
	void *dbuf = nullptr;
	CK(hipMalloc(&dbuf, 8 << 20));
	/* heap memory at a 16-byte phase, as numpy arrays sit */
	uint8_t *h = (uint8_t *)malloc(16 << 20);
	memset(h, 1, 16 << 20);
	uint8_t *p = (uint8_t *)(((uintptr_t)h + 4095) & ~(uintptr_t)4095) + 0x110;
	variant("A: heap, small 409664 then large 804288, no use", p, 409664, 804288, false, dbuf);
	variant("B: heap, small then large, DMA from the small one first", p + (4 << 20), 409664,
		804288, true, dbuf);
	/* page-aligned start */
	uint8_t *q = (uint8_t *)(((uintptr_t)h + (9 << 20) + 4095) & ~(uintptr_t)4095);
	variant("C: page-aligned start, small then large, DMA first", q, 409664, 804288, true, dbuf);
	/* mmap'd, locked and populated, like libxudp's anon_map (common.h:37-41) */
	void *m = mmap(nullptr, 4 << 20, PROT_READ | PROT_WRITE,
		       MAP_PRIVATE | MAP_ANONYMOUS | MAP_POPULATE | MAP_LOCKED, -1, 0);
	if (m != MAP_FAILED)
		variant("D: anon_map (MAP_LOCKED|MAP_POPULATE) + 0x110, DMA first",
			(uint8_t *)m + 0x110, 409664, 804288, true, dbuf);
	/* same size twice */
	variant("E: heap, same size twice, DMA first", p + (2 << 20), 409664, 409664, true, dbuf);
	CK(hipFree(dbuf));
	free(h);
	printf("reg_probe done\n");
	return 0;
}
