#!/usr/bin/env python3
"""Apply INTEGRATION.md sections 2-3 to a scratch copy of the reference's keyhunt.cpp and build it
against the engine: oracle/_ref/keyhunt_gpu.

This is the reference-side binding a keyhunt maintainer would add, compiled for real.  Nothing of the
reference is stored in this repository: the script reads /root/reference/keyhunt.cpp, inserts the
engine binding at three anchors (each must match exactly once, else the script fails), writes the
patched copy to a scratch directory and links it with the reference's own objects (built from its
sources by oracle/Makefile.ref) and keyhunt_amd/lib/libkh_gpu.so.  With KH_GPU=1 in the
environment the patched binary's workers hand their work to the GPU:

  thread_process      (keyhunt.cpp:3265-3861)  one kh_scan per N_SEQUENTIAL_MAX chunk taken from
                      the reference's own n_range_start cursor under write_random; hits printed by
                      the reference's own writekey / writekeyeth
  thread_process_bsgs (keyhunt.cpp:4549-4888)  kh_bsgs_setup/build + kh_bsgs_set_targets once, then
                      whole bases from the BSGS_CURRENT cursor under bsgs_thread, one kh_bsgs_scan per
                      batch; hits printed and recorded as keyhunt.cpp:4825-4858 does

Without KH_GPU the binary is the reference unchanged.  tests/test_gpu_integration.py runs it on
reference-CLI fixtures.  Usage: python integration/patch_reference.py [--ref /root/reference]
"""
import argparse
import os
import subprocess
import sys
import tempfile

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
OUT = os.path.join(REPO, "oracle", "_ref", "keyhunt_gpu")

BINDING = r'''
/* ---- MI355X engine binding (integration/patch_reference.py, INTEGRATION.md sections 2-3) ---- */
#include "kh_gpu.h"
static kh_ctx *kh_gpu_open(int thread_number) {
	int ndev = 0;
	kh_device_count(&ndev);
	kh_ctx *gpu = NULL;
	if (ndev < 1 || kh_open(thread_number % ndev, &gpu) != KH_OK) {
		fprintf(stderr, "[E] kh_open: no usable GPU\n");
		exit(EXIT_FAILURE);
	}
	return gpu;
}
static void kh_gpu_check(kh_ctx *gpu, int r, const char *what) {
	if (r != KH_OK) {
		fprintf(stderr, "[E] %s: %s (%s)\n", what, kh_strerror(r), kh_last_error(gpu));
		exit(EXIT_FAILURE);
	}
}
/* section 2: the address family, one kh_scan per chunk of the reference's own cursor */
void *kh_gpu_thread_process(void *vargp) {
	struct tothread *tt = (struct tothread *)vargp;
	int thread_number = tt->nt;
	free(tt);
	kh_ctx *gpu = kh_gpu_open(thread_number);
	kh_gpu_check(gpu, kh_set_targets(gpu, (const uint8_t *)addressTable, N, N), "kh_set_targets");
	uint8_t start_be[32], stride_be[32];
	stride.Get32Bytes(stride_be);
	std::vector<kh_hit> hits(1 << 16);
	uint32_t mode = FLAGMODE == MODE_XPOINT ? KH_MODE_XPOINT : (FLAGCRYPTO == CRYPTO_ETH ? KH_MODE_ETH : KH_MODE_ADDRESS);
	if (FLAGENDOMORPHISM) mode |= KH_MODE_ENDO;
	/* the reference numbers its search kinds the other way round (keyhunt.cpp:89-91) */
	const uint32_t search = FLAGSEARCH == SEARCH_COMPRESS ? KH_SEARCH_COMPRESS
	                      : FLAGSEARCH == SEARCH_UNCOMPRESS ? KH_SEARCH_UNCOMPRESS : KH_SEARCH_BOTH;
	Int key_mpz;
	for (;;) {
		pthread_mutex_lock(&write_random);
		const bool more = n_range_start.IsLower(&n_range_end);
		if (more) {
			key_mpz.Set(&n_range_start);
			n_range_start.Add(N_SEQUENTIAL_MAX);
		}
		pthread_mutex_unlock(&write_random);
		if (!more) break;
		key_mpz.Get32Bytes(start_be);
		uint32_t nh = 0;
		kh_gpu_check(gpu, kh_scan(gpu, start_be, stride_be, N_SEQUENTIAL_MAX, mode, search, hits.data(),
		                          (uint32_t)hits.size(), &nh), "kh_scan");
		for (uint32_t i = 0; i < nh; i++) {  /* confirmed by searchbinary, parity-fixed, in print order */
			Int k;
			k.Set32Bytes(hits[i].key);
			if ((hits[i].kind & 15) == KH_KIND_ETH)
				writekeyeth(&k);
			else
				writekey(hits[i].compressed != 0, &k);
		}
		steps[thread_number].fetch_add(N_SEQUENTIAL_MAX / 1024, std::memory_order_relaxed);
	}
	kh_close(gpu);
	ends[thread_number] = 1;
	return NULL;
}
/* section 3: BSGS, whole bases from the reference's BSGS_CURRENT cursor, one kh_bsgs_scan per batch */
void *kh_gpu_thread_process_bsgs(void *vargp) {
	struct tothread *tt = (struct tothread *)vargp;
	int thread_number = tt->nt;
	free(tt);
	kh_ctx *gpu = kh_gpu_open(thread_number);
	kh_bsgs_info info;
	kh_gpu_check(gpu, kh_bsgs_setup(gpu, BSGS_N.GetInt64(), (uint64_t)KFACTOR, &info), "kh_bsgs_setup");
	kh_gpu_check(gpu, kh_bsgs_build(gpu), "kh_bsgs_build");
	std::vector<uint8_t> xy(64 * (size_t)bsgs_point_number);
	for (uint32_t k = 0; k < bsgs_point_number; k++) {
		OriginalPointsBSGS[k].x.Get32Bytes(&xy[64 * k]);
		OriginalPointsBSGS[k].y.Get32Bytes(&xy[64 * k + 32]);
	}
	kh_gpu_check(gpu, kh_bsgs_set_targets(gpu, xy.data(), bsgs_point_number), "kh_bsgs_set_targets");
	const uint64_t per_call = (1ULL << 31) / (info.cycles * 1024) ? (1ULL << 31) / (info.cycles * 1024) : 1;
	std::vector<kh_bsgs_found> found(bsgs_point_number + 1);
	Int base_key;
	for (;;) {
		uint64_t nb = 0;
		pthread_mutex_lock(&bsgs_thread);
		base_key.Set(&BSGS_CURRENT);
		while (nb < per_call && BSGS_CURRENT.IsLower(&n_range_end)) {
			BSGS_CURRENT.Add(&BSGS_STEP);
			nb++;
		}
		pthread_mutex_unlock(&bsgs_thread);
		if (!nb) break;
		uint8_t st[32];
		base_key.Get32Bytes(st);
		uint32_t nf = 0;
		kh_gpu_check(gpu, kh_bsgs_scan(gpu, st, nb, found.data(), (uint32_t)found.size(), &nf), "kh_bsgs_scan");
		for (uint32_t i = 0; i < nf; i++) {
			const uint32_t t = found[i].target;
			if (bsgs_found[t]) continue;
			Int keyfound;
			keyfound.Set32Bytes(found[i].key);
			char *hextemp = keyfound.GetBase16();
			printf("[+] Thread Key found privkey %s   ", hextemp);
			Point point_found = secp->ComputePublicKey(&keyfound);
			char *aux_c = secp->GetPublicKeyHex(OriginalPointsBSGScompressed[t], point_found);
			printf("[+] Publickey %s\n", aux_c);
			pthread_mutex_lock(&write_keys);
			FILE *filekey = fopen("KEYFOUNDKEYFOUND.txt", "a");
			if (filekey != NULL) {
				fprintf(filekey, "Key found privkey %s\nPublickey %s\n", hextemp, aux_c);
				fclose(filekey);
			}
			pthread_mutex_unlock(&write_keys);
			free(hextemp);
			free(aux_c);
			bsgs_found[t] = 1;
			int all = 1;
			for (uint32_t l = 0; l < bsgs_point_number && all; l++) all &= bsgs_found[l];
			if (all) {
				printf("All points were found\n");
				exit(EXIT_FAILURE);
			}
		}
		steps[thread_number].fetch_add(2 * nb, std::memory_order_relaxed);
		bsgs_steps_total.fetch_add(2 * nb, std::memory_order_relaxed);
	}
	kh_close(gpu);
	ends[thread_number] = 1;
	return NULL;
}
/* ---- end of the engine binding ---- */

'''

# (anchor, replacement): each anchor must occur exactly once in keyhunt.cpp
EDITS = [
    # the binding's functions, right before thread_process's definition (keyhunt.cpp:3262)
    ("\n#if defined(_WIN64) && !defined(__CYGWIN__)\nDWORD WINAPI thread_process(LPVOID vargp) {\n",
     "\n" + BINDING + "#if defined(_WIN64) && !defined(__CYGWIN__)\nDWORD WINAPI thread_process(LPVOID vargp) {\n"),
    # dispatch at the top of thread_process (keyhunt.cpp:3265)
    ("void *thread_process(void *vargp)\t{\n#endif\n",
     "void *thread_process(void *vargp)\t{\n#endif\n\tif (getenv(\"KH_GPU\")) return kh_gpu_thread_process(vargp);\n"),
    # dispatch at the top of thread_process_bsgs (keyhunt.cpp:4549)
    ("void *thread_process_bsgs(void *vargp)\t{\n#endif\n",
     "void *thread_process_bsgs(void *vargp)\t{\n#endif\n\tif (getenv(\"KH_GPU\")) return kh_gpu_thread_process_bsgs(vargp);\n"),
]


def patch(src: str) -> str:
    for anchor, repl in EDITS:
        n = src.count(anchor)
        if n != 1:
            sys.exit(f"patch_reference: anchor found {n} times (expected once): {anchor!r}")
        src = src.replace(anchor, repl)
    return src


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--ref", default="/root/reference")
    ap.add_argument("--scratch", default=None, help="directory for the patched copy (default: a temp dir)")
    a = ap.parse_args()
    ref = a.ref
    if not os.path.isfile(os.path.join(ref, "keyhunt.cpp")):
        sys.exit(f"patch_reference: {ref}/keyhunt.cpp not found")
    jobs = str(min(16, os.cpu_count() or 8))
    subprocess.run(["make", "-s", "-C", os.path.join(REPO, "oracle"), "-f", "Makefile.ref", f"-j{jobs}", f"REF={ref}"],
                   check=True)
    lib = os.path.join(REPO, "keyhunt_amd", "lib", "libkh_gpu.so")
    if not os.path.exists(lib):
        sys.exit("patch_reference: build keyhunt_amd/lib/libkh_gpu.so first (make -C keyhunt_amd)")
    scratch = a.scratch or tempfile.mkdtemp(prefix="kh_integration_")
    os.makedirs(scratch, exist_ok=True)
    patched = os.path.join(scratch, "keyhunt_gpu.cpp")
    with open(os.path.join(ref, "keyhunt.cpp")) as f:
        src = patch(f.read())
    with open(patched, "w") as f:
        f.write(src)
    obj = os.path.join(REPO, "oracle", "_ref", "obj")
    objs = [os.path.join(obj, o) for o in ("Int.o", "Point.o", "SECP256K1.o", "IntMod.o", "Random.o", "IntGroup.o",
                                           "ripemd160.o", "sha256.o", "ripemd160_sse.o", "sha256_sse.o", "bloom.o",
                                           "xxhash.o", "oldbloom.o", "base58.o", "rmd160.o", "sha3.o", "keccak.o",
                                           "util.o")]
    cmd = ["g++", "-m64", "-march=x86-64-v3", "-mssse3", "-O3", "-w", f"-I{ref}", f"-I{os.path.join(REPO, 'include')}",
           "-o", OUT, patched] + objs + [f"-L{os.path.dirname(lib)}", "-lkh_gpu",
                                         "-Wl,-rpath,$ORIGIN/../../keyhunt_amd/lib", "-lm", "-lpthread"]
    subprocess.run(cmd, check=True)
    print(f"patch_reference: {OUT} (patched copy in {patched})")


if __name__ == "__main__":
    main()
