#!/usr/bin/env python3
"""Apply INTEGRATION.md sections 1-3 to a scratch copy of the reference's keyhunt.cpp and build it
against the engine: oracle/_ref/keyhunt_gpu.

This is the reference-side binding a keyhunt maintainer would add, compiled for real.  Nothing of the
reference is stored in this repository: the script reads /root/reference/keyhunt.cpp, inserts the
engine binding at six anchors (each must match exactly once, else the script fails), writes the
patched copy to a scratch directory and links it with the reference's own objects (built from its
sources by oracle/Makefile.ref) and keyhunt_amd/lib/libkh_gpu.so.  With KH_GPU=1 in the
environment the patched binary hands its work to the GPU, one engine context per device shared by
the worker threads of that device:

  BSGS tables         (keyhunt.cpp:1686-2697)  the bloom / bP-table allocation, the thread_bPload pool
                      and the -S file blocks are replaced by kh_bsgs_setup + kh_bsgs_load (the -S
                      files, when all four exist) or kh_bsgs_build (+ kh_bsgs_save with -S) per device,
                      for the sequential schedule with 2N-spaced bases without --mapped / --ptable
                      (other schedules keep the reference's CPU tables and workers)
  thread_process      (keyhunt.cpp:3265-3861)  one kh_scan per N_SEQUENTIAL_MAX chunk taken from
                      the reference's own n_range_start cursor under write_random; hits printed by
                      the reference's own writekey / writekeyeth
  thread_process_bsgs (keyhunt.cpp:4549-4888)  whole bases from the BSGS_CURRENT cursor under
                      bsgs_thread, one kh_bsgs_scan per batch; hits printed and recorded as
                      keyhunt.cpp:4825-4858 does

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
/* ---- MI355X engine binding (integration/patch_reference.py, INTEGRATION.md sections 1-3) ---- */
#include <chrono>
#include "kh_gpu.h"
/* Section 1: one engine context per device, shared by the worker threads of that device (thread t
   uses device t % ndev); calls on a context are serialised by its mutex (a kh_ctx is not
   re-entrant).  Contexts are opened on first use, or by kh_gpu_bsgs_tables in main. */
#define KH_GPU_MAXDEV 64
static int kh_gpu_ndev = 0;
static kh_ctx *kh_gpu_ctx[KH_GPU_MAXDEV];
static pthread_mutex_t kh_gpu_ctx_mutex[KH_GPU_MAXDEV];
static pthread_mutex_t kh_gpu_open_mutex = PTHREAD_MUTEX_INITIALIZER;
static int kh_gpu_bsgs_ready = 0;  /* BSGS tables are in every device's HBM (kh_gpu_bsgs_tables) */
static void kh_gpu_check(kh_ctx *gpu, int r, const char *what) {
	if (r != KH_OK) {
		fprintf(stderr, "[E] %s: %s (%s)\n", what, kh_strerror(r), gpu ? kh_last_error(gpu) : "");
		exit(EXIT_FAILURE);
	}
}
/* the device count; opens nothing (call with kh_gpu_open_mutex held, or before the threads start) */
static int kh_gpu_devices(void) {
	if (!kh_gpu_ndev) {
		int n = 0;
		kh_device_count(&n);
		if (n < 1) {
			fprintf(stderr, "[E] kh_open: no usable GPU\n");
			exit(EXIT_FAILURE);
		}
		kh_gpu_ndev = n < KH_GPU_MAXDEV ? n : KH_GPU_MAXDEV;
		for (int d = 0; d < kh_gpu_ndev; d++) pthread_mutex_init(&kh_gpu_ctx_mutex[d], NULL);
	}
	return kh_gpu_ndev;
}
/* the context of device d, opened on first use; `fresh` tells the caller to load it (targets) */
static kh_ctx *kh_gpu_open_dev(int d, bool *fresh) {
	*fresh = false;
	if (!kh_gpu_ctx[d]) {
		kh_gpu_check(NULL, kh_open(d, &kh_gpu_ctx[d]), "kh_open");
		*fresh = true;
	}
	return kh_gpu_ctx[d];
}
/* section 2: the address family, one kh_scan per chunk of the reference's own cursor */
void *kh_gpu_thread_process(void *vargp) {
	struct tothread *tt = (struct tothread *)vargp;
	int thread_number = tt->nt;
	free(tt);
	pthread_mutex_lock(&kh_gpu_open_mutex);
	const int dev = thread_number % kh_gpu_devices();
	bool fresh;
	kh_ctx *gpu = kh_gpu_open_dev(dev, &fresh);
	/* -m rmd160 --rmd-batch-size (keyhunt.cpp:3301-3307): the reference's groups of that size */
	const uint32_t group = FLAGMODE == MODE_RMD160 ? (uint32_t)rmd_batch_size : CPU_GRP_SIZE;
	if (fresh) {  /* the first thread of this device loads its targets */
		kh_gpu_check(gpu, kh_set_targets(gpu, (const uint8_t *)addressTable, N, N), "kh_set_targets");
		kh_gpu_check(gpu, kh_set_rmd_batch(gpu, group), "kh_set_rmd_batch");
	}
	pthread_mutex_unlock(&kh_gpu_open_mutex);
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
		pthread_mutex_lock(&kh_gpu_ctx_mutex[dev]);
		const int r = kh_scan(gpu, start_be, stride_be, N_SEQUENTIAL_MAX, mode, search, hits.data(),
		                      (uint32_t)hits.size(), &nh);
		pthread_mutex_unlock(&kh_gpu_ctx_mutex[dev]);
		kh_gpu_check(gpu, r, "kh_scan");
		for (uint32_t i = 0; i < nh; i++) {  /* confirmed by searchbinary, parity-fixed, in print order */
			Int k;
			k.Set32Bytes(hits[i].key);
			if ((hits[i].kind & 15) == KH_KIND_ETH)
				writekeyeth(&k);
			else
				writekey(hits[i].compressed != 0, &k);
		}
		steps[thread_number].fetch_add((N_SEQUENTIAL_MAX + group - 1) / group, std::memory_order_relaxed);  /* one per group */
	}
	ends[thread_number] = 1;
	return NULL;
}
/* section 3, setup: the engine's tables replace the reference's bloom / bP-table allocation, the
   thread_bPload pool and the -S file blocks (keyhunt.cpp:1686-2697) for the sequential schedule with
   2N-spaced bases.  Every device gets its own replica: read from the -S files when all four are
   there (kh_bsgs_load, the reference's own format and checksums), else built on the GPU and, with
   -S, written by device 0 (kh_bsgs_save). */
static bool kh_gpu_bsgs_wanted(void) {
	return getenv("KH_GPU") && FLAGBSGSMODE == 0 && BSGS_STEP.IsEqual(&BSGS_N_double) && !FLAGMAPPED &&
	       !bptable_filename && !FLAGLOADPTABLE;
}
static void kh_gpu_bsgs_tables(void) {
	const auto t0 = std::chrono::steady_clock::now();
	const int ndev = kh_gpu_devices();
	const int used = NTHREADS < ndev ? NTHREADS : ndev;
	std::vector<uint8_t> xy(64 * (size_t)bsgs_point_number);
	for (uint32_t k = 0; k < bsgs_point_number; k++) {
		OriginalPointsBSGS[k].x.Get32Bytes(&xy[64 * k]);
		OriginalPointsBSGS[k].y.Get32Bytes(&xy[64 * k + 32]);
	}
	int loaded = 0;
	for (int d = 0; d < used; d++) {
		bool fresh;
		kh_ctx *gpu = kh_gpu_open_dev(d, &fresh);
		kh_bsgs_info info;
		kh_gpu_check(gpu, kh_bsgs_set_bloom_multiplier(gpu, (uint32_t)FLAGBLOOMMULTIPLIER), "kh_bsgs_set_bloom_multiplier");
		kh_gpu_check(gpu, kh_bsgs_setup(gpu, BSGS_N.GetInt64(), (uint64_t)KFACTOR, &info), "kh_bsgs_setup");
		int r = KH_E_IO;
		if (FLAGSAVEREADFILE) r = kh_bsgs_load(gpu, ".", FLAGSKIPCHECKSUM ? KH_LOAD_SKIP_CHECKSUM : 0);
		if (r == KH_E_IO) {
			kh_gpu_check(gpu, kh_bsgs_build(gpu), "kh_bsgs_build");
			if (FLAGSAVEREADFILE && d == 0) kh_gpu_check(gpu, kh_bsgs_save(gpu, "."), "kh_bsgs_save");
		} else {
			kh_gpu_check(gpu, r, "kh_bsgs_load");
			loaded++;
		}
		kh_gpu_check(gpu, kh_bsgs_set_targets(gpu, xy.data(), bsgs_point_number), "kh_bsgs_set_targets");
	}
	const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
	printf("[+] MI355X engine: bloom filters and bP table for %" PRIu64 " baby steps %s on %d GPU(s) in %.2f s\n",
	       bsgs_m, loaded == used ? "read from the -S files" : "built", used, secs);
	fflush(stdout);
	kh_gpu_bsgs_ready = 1;
}
/* section 3, worker: whole bases from the reference's BSGS_CURRENT cursor, one kh_bsgs_scan per batch
   on the shared context of the thread's device */
void *kh_gpu_thread_process_bsgs(void *vargp) {
	struct tothread *tt = (struct tothread *)vargp;
	int thread_number = tt->nt;
	free(tt);
	const int dev = thread_number % kh_gpu_ndev;
	kh_ctx *gpu = kh_gpu_ctx[dev];
	if (!gpu) {  /* more devices than threads cannot happen (used = min(NTHREADS, ndev)) */
		ends[thread_number] = 1;
		return NULL;
	}
	const uint64_t per_call = (1ULL << 31) / (bsgs_aux ? bsgs_aux : 1) ? (1ULL << 31) / (bsgs_aux ? bsgs_aux : 1) : 1;
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
		pthread_mutex_lock(&kh_gpu_ctx_mutex[dev]);
		const int r = kh_bsgs_scan(gpu, st, nb, found.data(), (uint32_t)found.size(), &nf);
		pthread_mutex_unlock(&kh_gpu_ctx_mutex[dev]);
		kh_gpu_check(gpu, r, "kh_bsgs_scan");
		for (uint32_t i = 0; i < nf; i++) {
			const uint32_t t = found[i].target;
			pthread_mutex_lock(&write_keys);
			if (bsgs_found[t]) {
				pthread_mutex_unlock(&write_keys);
				continue;
			}
			bsgs_found[t] = 1;
			Int keyfound;
			keyfound.Set32Bytes(found[i].key);
			char *hextemp = keyfound.GetBase16();
			printf("[+] Thread Key found privkey %s   ", hextemp);
			Point point_found = secp->ComputePublicKey(&keyfound);
			char *aux_c = secp->GetPublicKeyHex(OriginalPointsBSGScompressed[t], point_found);
			printf("[+] Publickey %s\n", aux_c);
			FILE *filekey = fopen("KEYFOUNDKEYFOUND.txt", "a");
			if (filekey != NULL) {
				fprintf(filekey, "Key found privkey %s\nPublickey %s\n", hextemp, aux_c);
				fclose(filekey);
			}
			free(hextemp);
			free(aux_c);
			int all = 1;
			for (uint32_t l = 0; l < bsgs_point_number && all; l++) all &= bsgs_found[l];
			pthread_mutex_unlock(&write_keys);
			if (all) {
				/* keyhunt.cpp:4811-4814; first wait until no other thread is inside the engine, so
				   that exit() does not tear the HIP runtime down under a running call */
				for (int d = 0; d < kh_gpu_ndev; d++) pthread_mutex_lock(&kh_gpu_ctx_mutex[d]);
				printf("All points were found\n");
				exit(EXIT_FAILURE);
			}
		}
		steps[thread_number].fetch_add(2 * nb, std::memory_order_relaxed);
		bsgs_steps_total.fetch_add(2 * nb, std::memory_order_relaxed);
	}
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
    # their prototypes before main (the table seam below is in main, keyhunt.cpp:664)
    ("\nint main(int argc, char **argv)\t{\n",
     "\nstatic bool kh_gpu_bsgs_wanted(void);\nstatic void kh_gpu_bsgs_tables(void);\n"
     "\nint main(int argc, char **argv)\t{\n"),
    # the table seam: the engine's tables instead of the reference's bloom / bP-table allocation,
    # thread_bPload pool and -S file blocks (keyhunt.cpp:1686-2697)
    ('\n                printf("[+] Bloom filter for %" PRIu64 " elements ",bsgs_m);\n',
     '\n\t\tif (kh_gpu_bsgs_wanted()) kh_gpu_bsgs_tables(); else {\n'
     '                printf("[+] Bloom filter for %" PRIu64 " elements ",bsgs_m);\n'),
    ("                if(!FLAGREADEDFILE4) FLAGREADEDFILE4 = 1;\n\t\ti = 0;\n\n\t\tbsgs_steps_total.store(0);\n",
     "                if(!FLAGREADEDFILE4) FLAGREADEDFILE4 = 1;\n\t\t}  /* end of the reference's CPU tables */\n"
     "\t\ti = 0;\n\n\t\tbsgs_steps_total.store(0);\n"),
    # dispatch at the top of thread_process (keyhunt.cpp:3265)
    ("void *thread_process(void *vargp)\t{\n#endif\n",
     "void *thread_process(void *vargp)\t{\n#endif\n\tif (getenv(\"KH_GPU\")) return kh_gpu_thread_process(vargp);\n"),
    # dispatch at the top of thread_process_bsgs (keyhunt.cpp:4549): only when the engine holds the tables
    ("void *thread_process_bsgs(void *vargp)\t{\n#endif\n",
     "void *thread_process_bsgs(void *vargp)\t{\n#endif\n\tif (kh_gpu_bsgs_ready) return kh_gpu_thread_process_bsgs(vargp);\n"),
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
