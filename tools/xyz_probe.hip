// xyz_probe.hip -- tuning tool (not product code): the memory access pattern of
// the one-pass 3-D step at 512^3, bs 2, in the product's device layout
// (gcmx.hip: row 544 doubles, 516 x 516 planes, 9 component planes per layer),
// with trivial arithmetic, to separate the access pattern's own time from the
// kernel's arithmetic.  Variants (VEC = doubles per lane, PL = x planes per block):
//   copy    : 9 loads + 9 stores per node (the compulsory 144 B/node)
//   xpat    : the fused kernel's loads (6 components at 5 x-planes + 3 at the
//             node: 33 loads) + 9 stores, marching y
//   xpat_ns : xpat without stores
//   xtx<TX> : xpat with TX adjacent x planes per thread (loads TX+4 planes)
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/xyz_probe tools/xyz_probe.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <ctime>

#define CK(x)                                                                           \
	do {                                                                                \
		hipError_t e = (x);                                                             \
		if (e != hipSuccess) {                                                          \
			std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e));                 \
			std::exit(1);                                                               \
		}                                                                               \
	} while (0)

constexpr int N = 512, BS = 2, ROW = 544, LEAD = 14;
constexpr long long STY = ROW, STX = (long long)ROW * (N + 2 * BS);
constexpr long long CS = ((STX * (N + 2 * BS)) + 63) / 64 * 64;
constexpr long long ORIGIN = LEAD + BS + BS * STY + BS * STX;

template <int VEC> struct V;
template <> struct V<1> {
	typedef double T;
	static __device__ double sum(T a) { return a; }
};
typedef double d2 __attribute__((ext_vector_type(2)));
template <> struct V<2> {
	typedef d2 T;
	static __device__ double sum(T a) { return a.x + a.y; }
};
template <int VEC>
__device__ __forceinline__ typename V<VEC>::T add(typename V<VEC>::T a, typename V<VEC>::T b) {
	if constexpr (VEC == 1) return a + b;
	else return a + b;
}

// MODE 0 copy, 1 xpat, 2 xpat no stores
template <int MODE, int VEC, int PL>
__global__ __launch_bounds__(512 / VEC * PL) void k_probe(const double* __restrict__ in,
                                                          double* __restrict__ out, int chunk) {
	typedef typename V<VEC>::T T;
	constexpr int LANES = 512 / VEC;
	const int z = (threadIdx.x % LANES) * VEC, sub = threadIdx.x / LANES;
	const int T_ = gridDim.x, b = blockIdx.x;
	const int p = (T_ % 8 == 0) ? (b % 8) * (T_ / 8) + b / 8 : b;
	const int np = N / PL;
	const int x = (p % np) * PL + sub, yb = (p / np) * chunk;
	const unsigned base = (unsigned)(ORIGIN + x * STX + z);
	double acc = 0;
	auto ld = [&](int c, unsigned o) { return *reinterpret_cast<const T*>(in + c * CS + o); };
	for (int y = yb; y < yb + chunk; y++) {
		const unsigned o = base + (unsigned)y * (unsigned)STY;
		T v[9];
		if constexpr (MODE == 0) {
#pragma unroll
			for (int c = 0; c < 9; c++) v[c] = ld(c, o);
		} else {
#pragma unroll
			for (int c = 0; c < 9; c++) {
				T s = ld(c, o);
				if (c < 6) {
#pragma unroll
					for (int k = -BS; k <= BS; k++)
						if (k != 0) s = add<VEC>(s, ld(c, o + (unsigned)(k * STX)));
				}
				v[c] = s;
			}
		}
		if constexpr (MODE == 2) {
#pragma unroll
			for (int c = 0; c < 9; c++) acc += V<VEC>::sum(v[c]);
		} else {
#pragma unroll
			for (int c = 0; c < 9; c++)
				__builtin_nontemporal_store(v[c], reinterpret_cast<T*>(out + c * CS + o));
		}
	}
	if (MODE == 2 && acc == 1234.5) out[0] = acc;
}

// Each thread: TX adjacent planes at one z; 6 components at TX+4 planes, 3 at the TX nodes.
// BAR: the fused kernel's Z exchange per row -- two barriers around 12 LDS row
// writes (6 components x 2 nodes), then 4 neighbour reads per component.
// ZT < 512: a block covers z [zp*ZT, zp*ZT + ZT) of the row (one wave per SIMD
// at one block per CU: the VGPR budget of a 512-register lane).
template <int TX, bool STORE, int KOPS = 0, bool BAR = false, int ZT = 512>
__global__ __launch_bounds__(ZT, ZT == 512 ? 2 : 1) void k_probe_tx(const double* __restrict__ in,
                                                     double* __restrict__ out, int chunk) {
	extern __shared__ double dyn_lds[];
	__shared__ double zl[BAR ? TX : 1][6][BAR ? 516 : 1];
	constexpr int NZ = 512 / ZT;
	if (threadIdx.x == 1023) dyn_lds[0] = 0.0;  // never true: keeps the dynamic LDS request
	const int T_ = gridDim.x, b = blockIdx.x;
	const int p0 = (T_ % 8 == 0) ? (b % 8) * (T_ / 8) + b / 8 : b;
	const int z = threadIdx.x + (p0 % NZ) * ZT, p = p0 / NZ;
	const int np = N / TX;
	const int x = (p % np) * TX, yb = (p / np) * chunk;
	const unsigned base = (unsigned)(ORIGIN + x * STX + z);
	double acc = 0;
	for (int y = yb; y < yb + chunk; y++) {
		const unsigned o = base + (unsigned)y * (unsigned)STY;
		double v[TX][9];
#pragma unroll
		for (int c = 0; c < 9; c++) {
			if (c < 6) {
				double w[TX + 4];
#pragma unroll
				for (int k = 0; k < TX + 4; k++) w[k] = in[c * CS + (long long)(o + (unsigned)((k - BS) * STX))];
#pragma unroll
				for (int t = 0; t < TX; t++) v[t][c] = w[t] + w[t + 1] + w[t + 2] + w[t + 3] + w[t + 4];
			} else {
#pragma unroll
				for (int t = 0; t < TX; t++) v[t][c] = in[c * CS + (long long)(o + (unsigned)(t * STX))];
			}
		}
		if constexpr (KOPS > 0) {  // KOPS fp64 add/mul per node, 9 independent chains
#pragma unroll
			for (int t = 0; t < TX; t++)
#pragma unroll 1
				for (int k = 0; k < KOPS / 18; k++)
#pragma unroll
					for (int c = 0; c < 9; c++) v[t][c] = v[t][c] * 0.999 + 0.001;
		}
		if constexpr (BAR) {
			__syncthreads();
#pragma unroll
			for (int t = 0; t < TX; t++)
#pragma unroll
				for (int c = 0; c < 6; c++) zl[t][c][2 + z] = v[t][c];
			__syncthreads();
#pragma unroll
			for (int t = 0; t < TX; t++)
#pragma unroll
				for (int c = 0; c < 6; c++)
					v[t][c] += (zl[t][c][z] + zl[t][c][z + 1]) + (zl[t][c][z + 3] + zl[t][c][z + 4]);
		}
#pragma unroll
		for (int t = 0; t < TX; t++)
#pragma unroll
			for (int c = 0; c < 9; c++) {
				if (STORE) __builtin_nontemporal_store(v[t][c], out + c * CS + (long long)(o + (unsigned)(t * STX)));
				else acc += v[t][c];
			}
	}
	if (!STORE && acc == 1234.5) out[0] = acc;
}

// x-marching: a block is a tile of TYB = TY + 2*BS y rows
// (one wave each) x 64 z lanes, marching x over XC planes.  Each lane keeps the
// X window (planes x-BS..x+BS of the 6 window components) in registers and loads
// ONE new plane per x step (6 window + 3 node-only components: 9 loads); the X
// results go to LDS, the Y stage of the TY inner rows reads rows y-BS..y+BS from
// LDS, the Z stage reads z-BS..z+BS of the Y results from LDS, and the 60 inner
// lanes of the TY inner rows store (z tiles overlap by 2*BS columns: the X and Y
// stages of the halo rows / columns are recomputed, the stores start at
// unaligned 60-column offsets).  Loads per stored node: 9 * TYB/TY * 64/60 plus
// the 2*BS-plane x prologue per chunk.  Trivial arithmetic.
template <int TY, int XC>
__global__ __launch_bounds__(64 * (TY + 2 * BS)) void k_probe_xm(const double* __restrict__ in,
                                                                 double* __restrict__ out) {
	constexpr int TYB = TY + 2 * BS, ZO = 64 - 2 * BS, W = 2 * BS + 1;
	__shared__ double xs[6][TYB][64];
	__shared__ double ys[6][TY][64];
	const int lane = threadIdx.x & 63, row = threadIdx.x >> 6;
	const int ntz = (N + ZO - 1) / ZO, nty = (N + TY - 1) / TY;
	const int b = blockIdx.x;
	const int tz = b % ntz, ty = (b / ntz) % nty, tx = b / (ntz * nty);
	const int z = tz * ZO - BS + lane, y = ty * TY - BS + row, x0 = tx * XC;
	const bool zin = z >= 0 && z < N, yin = y >= 0 && y < N;
	const int zc = zin ? z : (z < 0 ? 0 : N - 1), yc = yin ? y : (y < 0 ? 0 : N - 1);
	const long long col = ORIGIN + (long long)yc * STY + zc;
	double win[6][W];
#pragma unroll
	for (int k = 0; k < W - 1; k++)  // prologue: planes x0-BS .. x0+BS-1
#pragma unroll
		for (int c = 0; c < 6; c++) win[c][k + 1] = in[c * CS + col + (long long)(x0 - BS + k) * STX];
	for (int x = x0; x < x0 + XC; x++) {
#pragma unroll
		for (int c = 0; c < 6; c++) {
#pragma unroll
			for (int k = 0; k < W - 1; k++) win[c][k] = win[c][k + 1];
			win[c][W - 1] = in[c * CS + col + (long long)(x + BS) * STX];
		}
		double node[3];
#pragma unroll
		for (int c = 0; c < 3; c++) node[c] = in[(6 + c) * CS + col + (long long)x * STX];
		__syncthreads();
#pragma unroll
		for (int c = 0; c < 6; c++) {
			double s = 0;
#pragma unroll
			for (int k = 0; k < W; k++) s += win[c][k];
			xs[c][row][lane] = s;
		}
		__syncthreads();
		const bool inner_row = row >= BS && row < BS + TY;
		double yv[6];
		if (inner_row) {
#pragma unroll
			for (int c = 0; c < 6; c++) {
				double s = 0;
#pragma unroll
				for (int k = -BS; k <= BS; k++) s += xs[c][row + k][lane];
				yv[c] = s;
				ys[c][row - BS][lane] = s;
			}
		}
		__syncthreads();
		const bool store = inner_row && lane >= BS && lane < 64 - BS && zin && yin;
		if (store) {
			const long long o = col + (long long)x * STX;
#pragma unroll
			for (int c = 0; c < 6; c++) {
				double s = yv[c];
#pragma unroll
				for (int k = -BS; k <= BS; k++)
					if (k) s += ys[c][row - BS][lane + k];
				__builtin_nontemporal_store(s, out + c * CS + o);
			}
#pragma unroll
			for (int c = 0; c < 3; c++) __builtin_nontemporal_store(node[c], out + (6 + c) * CS + o);
		}
	}
}


// Generalised two/four-plane pattern (VERDICT r4 item 1 follow-up): ZT threads
// per block, each lane holding ZR groups of VEC adjacent z columns (VEC = 2:
// 16-byte loads) at TX adjacent x planes; a block covers ZT * ZR * VEC columns
// of a row.  One block per CU when launched with 96 KB of dynamic LDS.
template <int TX, int KOPS, int ZT, int ZR, int VEC>
__global__ __launch_bounds__(ZT, ZT == 512 ? 2 : 1) void k_probe_tz(const double* __restrict__ in,
                                                                   double* __restrict__ out, int chunk) {
	typedef typename V<VEC>::T T;
	extern __shared__ double dyn_lds[];
	constexpr int ZB = ZT * ZR * VEC, NZ = 512 / ZB;
	if (threadIdx.x == 1023) dyn_lds[0] = 0.0;
	const int T_ = gridDim.x, b = blockIdx.x;
	const int p0 = (T_ % 8 == 0) ? (b % 8) * (T_ / 8) + b / 8 : b;
	const int zb = (p0 % NZ) * ZB, p = p0 / NZ;
	const int np = N / TX;
	const int x = (p % np) * TX, yb = (p / np) * chunk;
	auto ld = [&](int c, long long o) { return *reinterpret_cast<const T*>(in + c * CS + o); };
	for (int y = yb; y < yb + chunk; y++) {
#pragma unroll
		for (int r = 0; r < ZR; r++) {
			const int z = zb + r * ZT * VEC + (int)threadIdx.x * VEC;
			const long long o = ORIGIN + x * STX + (long long)y * STY + z;
			T v[TX][9];
#pragma unroll
			for (int c = 0; c < 9; c++) {
				if (c < 6) {
					T w[TX + 4];
#pragma unroll
					for (int k = 0; k < TX + 4; k++) w[k] = ld(c, o + (long long)(k - BS) * STX);
#pragma unroll
					for (int t = 0; t < TX; t++) v[t][c] = w[t] + w[t + 1] + w[t + 2] + w[t + 3] + w[t + 4];
				} else {
#pragma unroll
					for (int t = 0; t < TX; t++) v[t][c] = ld(c, o + (long long)t * STX);
				}
			}
			if constexpr (KOPS > 0) {
#pragma unroll
				for (int t = 0; t < TX; t++)
#pragma unroll 1
					for (int k = 0; k < KOPS / 18; k++)
#pragma unroll
						for (int c = 0; c < 9; c++) v[t][c] = v[t][c] * 0.999 + 0.001;
			}
#pragma unroll
			for (int t = 0; t < TX; t++)
#pragma unroll
				for (int c = 0; c < 9; c++)
					__builtin_nontemporal_store(v[t][c], reinterpret_cast<T*>(out + c * CS + o + (long long)t * STX));
		}
	}
}

template <int TX, int KOPS, int ZT, int ZR, int VEC>
void tz(const double* in, double* out, int chunk, size_t shm) {
	const double nodes = (double)N * N * N;
	constexpr int ZB = ZT * ZR * VEC;
	dim3 grid((N / chunk) * (N / TX) * (512 / ZB));
	hipEvent_t a, b;
	CK(hipEventCreate(&a));
	CK(hipEventCreate(&b));
	// PROBE_REPS (default 10) timed launches; the CLOCK_MONOTONIC span of the
	// timed launches is printed so that a power sampler (tools/power_probe.py)
	// can attribute its samples to the variant
	static const int reps = std::getenv("PROBE_REPS") ? std::atoi(std::getenv("PROBE_REPS")) : 10;
	hipLaunchKernelGGL((k_probe_tz<TX, KOPS, ZT, ZR, VEC>), grid, dim3(ZT), shm, 0, in, out, chunk);
	CK(hipDeviceSynchronize());
	timespec t0, t1;
	clock_gettime(CLOCK_MONOTONIC, &t0);
	CK(hipEventRecord(a));
	for (int r = 0; r < reps; r++)
		hipLaunchKernelGGL((k_probe_tz<TX, KOPS, ZT, ZR, VEC>), grid, dim3(ZT), shm, 0, in, out, chunk);
	CK(hipEventRecord(b));
	CK(hipEventSynchronize(b));
	clock_gettime(CLOCK_MONOTONIC, &t1);
	float ms = 0;
	CK(hipEventElapsedTime(&ms, a, b));
	ms /= reps;
	std::printf("TZ: %d planes x %d z-groups x %d adjacent z per lane, %d threads/block%s, chunk %3d, + %d fp64 ops/node: "
	            "%.3f ms (%.0f GB/s) [mono %.6f %.6f]\n",
	            TX, ZR, VEC, ZT, shm ? " (1 block/CU)" : "", chunk, KOPS, ms, 144.0 * nodes / (ms * 1e6),
	            t0.tv_sec + 1e-9 * t0.tv_nsec, t1.tv_sec + 1e-9 * t1.tv_nsec);
	std::fflush(stdout);
}


// Box characterisation: an fp64-FMA-only kernel on random
// operands, no memory traffic in the loop -- the clock a box holds when the VALU
// alone draws the power.  Eight independent chains per lane, ITERS iterations;
// 4 cycles per wave64 fp64 FMA per SIMD, so the effective clock is
// (waves per SIMD x ITERS x 8 x 4 cycles) / time.
template <int ITERS>
__global__ __launch_bounds__(256) void k_valu_fp64(double* __restrict__ out, unsigned long long seed) {
	unsigned long long s = seed ^ (0x9E3779B97F4A7C15ull * (blockIdx.x * 256 + threadIdx.x + 1));
	double a[8], b[8];
#pragma unroll
	for (int i = 0; i < 8; i++) {
		s = s * 6364136223846793005ull + 1442695040888963407ull;
		a[i] = 0.5 + (double)(s >> 11) * 0x1.0p-54;
		b[i] = 1.0 - (double)((s >> 7) & 0xffff) * 0x1.0p-20;
	}
	const double c = 0.999999 + (double)(s & 0xff) * 1e-12;
	for (int k = 0; k < ITERS; k++) {
#pragma unroll
		for (int i = 0; i < 8; i++) a[i] = __builtin_fma(a[i], b[i], c * 1e-3);
	}
	double acc = 0;
#pragma unroll
	for (int i = 0; i < 8; i++) acc += a[i];
	if (acc == 1234.5) out[0] = acc;
}

void valu_span(double* out, int cus) {
	constexpr int ITERS = 1 << 16;
	static const int reps = std::getenv("PROBE_REPS") ? std::atoi(std::getenv("PROBE_REPS")) : 10;
	const int blocks = cus * 8;  // 8 waves per SIMD... 8 blocks of 4 waves per CU
	hipEvent_t a, b;
	CK(hipEventCreate(&a));
	CK(hipEventCreate(&b));
	hipLaunchKernelGGL((k_valu_fp64<ITERS>), dim3(blocks), dim3(256), 0, 0, out, 1ull);
	CK(hipDeviceSynchronize());
	timespec t0, t1;
	clock_gettime(CLOCK_MONOTONIC, &t0);
	CK(hipEventRecord(a));
	for (int r = 0; r < reps; r++) hipLaunchKernelGGL((k_valu_fp64<ITERS>), dim3(blocks), dim3(256), 0, 0, out, 2ull + r);
	CK(hipEventRecord(b));
	CK(hipEventSynchronize(b));
	clock_gettime(CLOCK_MONOTONIC, &t1);
	float ms = 0;
	CK(hipEventElapsedTime(&ms, a, b));
	ms /= reps;
	// per SIMD: 8 waves (8 blocks x 4 waves / 4 SIMDs) x ITERS x 8 FMAs x 4 cycles
	const double cycles = 8.0 * ITERS * 8 * 4;
	std::printf("fp64 FMA only (8 waves/SIMD, random operands): %.3f ms, effective clock %.0f MHz "
	            "[mono %.6f %.6f]\n", ms, cycles / (ms * 1e-3) / 1e6, t0.tv_sec + 1e-9 * t0.tv_nsec,
	            t1.tv_sec + 1e-9 * t1.tv_nsec);
	std::fflush(stdout);
}

// the flat 16-B copy of the layout (k_probe MODE 0, VEC 2) with its monotonic span
void copy_span(const double* in, double* out) {
	const double nodes = (double)N * N * N;
	static const int reps = std::getenv("PROBE_REPS") ? std::atoi(std::getenv("PROBE_REPS")) : 10;
	dim3 grid((N / 128) * N), block(256);
	hipEvent_t a, b;
	CK(hipEventCreate(&a));
	CK(hipEventCreate(&b));
	hipLaunchKernelGGL((k_probe<0, 2, 1>), grid, block, 0, 0, in, out, 128);
	CK(hipDeviceSynchronize());
	timespec t0, t1;
	clock_gettime(CLOCK_MONOTONIC, &t0);
	CK(hipEventRecord(a));
	for (int r = 0; r < reps; r++) hipLaunchKernelGGL((k_probe<0, 2, 1>), grid, block, 0, 0, in, out, 128);
	CK(hipEventRecord(b));
	CK(hipEventSynchronize(b));
	clock_gettime(CLOCK_MONOTONIC, &t1);
	float ms = 0;
	CK(hipEventElapsedTime(&ms, a, b));
	ms /= reps;
	std::printf("copy (16-B lanes, layout planes): %.3f ms (%.0f GB/s) [mono %.6f %.6f]\n", ms,
	            144.0 * nodes / (ms * 1e6), t0.tv_sec + 1e-9 * t0.tv_nsec, t1.tv_sec + 1e-9 * t1.tv_nsec);
	std::fflush(stdout);
}

template <int TY, int XC>
void xmarch(const double* in, double* out) {
	const double nodes = (double)N * N * N;
	constexpr int ZO = 64 - 2 * BS;
	const int ntz = (N + ZO - 1) / ZO, nty = (N + TY - 1) / TY;
	dim3 grid(ntz * nty * (N / XC));
	hipEvent_t a, b;
	CK(hipEventCreate(&a));
	CK(hipEventCreate(&b));
	for (int r = 0; r < 11; r++) {
		if (r == 1) CK(hipEventRecord(a));
		hipLaunchKernelGGL((k_probe_xm<TY, XC>), grid, dim3(64 * (TY + 2 * BS)), 0, 0, in, out);
	}
	CK(hipEventRecord(b));
	CK(hipEventSynchronize(b));
	float ms = 0;
	CK(hipEventElapsedTime(&ms, a, b));
	ms /= 10;
	const double loads = 9.0 * (TY + 2 * BS) / TY * 64.0 / ZO * (XC + 2.0 * BS * 6.0 / 9.0) / XC;
	std::printf("x-march TY %2d (+%d halo rows) XC %3d: %.2f loads/node: %.3f ms (%.0f GB/s)\n", TY, 2 * BS, XC,
	            loads, ms, 144.0 * nodes / (ms * 1e6));
}

template <int TX, int KOPS, bool BAR = false, int ZT = 512>
void ops_tx(const double* in, double* out, int chunk, size_t shm = 0) {
	const double nodes = (double)N * N * N;
	dim3 grid((N / chunk) * (N / TX) * (512 / ZT));
	hipEvent_t a, b;
	CK(hipEventCreate(&a));
	CK(hipEventCreate(&b));
	for (int r = 0; r < 11; r++) {
		if (r == 1) CK(hipEventRecord(a));
		hipLaunchKernelGGL((k_probe_tx<TX, true, KOPS, BAR, ZT>), grid, dim3(ZT), shm, 0, in, out, chunk);
	}
	CK(hipEventRecord(b));
	CK(hipEventSynchronize(b));
	float ms = 0;
	CK(hipEventElapsedTime(&ms, a, b));
	ms /= 10;
	std::printf("TX %d planes/thread chunk %3d + %d fp64 ops/node%s%s%s: %.3f ms (%.0f GB/s)\n", TX, chunk, KOPS,
	            BAR ? " + Z exchange (2 barriers/row)" : "", shm ? " (1 block/CU)" : "",
	            ZT == 512 ? "" : ZT == 256 ? " (256-thread blocks: 1 wave/SIMD)" : " (ZT?)", ms,
	            144.0 * nodes / (ms * 1e6));
}

template <int TX>
void family_tx(const double* in, double* out, int chunk) {
	const double nodes = (double)N * N * N;
	float t[2];
	for (int m = 0; m < 2; m++) {
		dim3 grid((N / chunk) * (N / TX));
		hipEvent_t a, b;
		CK(hipEventCreate(&a));
		CK(hipEventCreate(&b));
		for (int r = 0; r < 11; r++) {
			if (r == 1) CK(hipEventRecord(a));
			if (m == 0) hipLaunchKernelGGL((k_probe_tx<TX, true>), grid, dim3(512), 0, 0, in, out, chunk);
			else hipLaunchKernelGGL((k_probe_tx<TX, false>), grid, dim3(512), 0, 0, in, out, chunk);
		}
		CK(hipEventRecord(b));
		CK(hipEventSynchronize(b));
		float ms = 0;
		CK(hipEventElapsedTime(&ms, a, b));
		t[m] = ms / 10;
	}
	std::printf("TX %d planes/thread chunk %3d: xpat %.3f ms (%.0f GB/s)  xpat_ns %.3f ms\n", TX, chunk,
	            t[0], 144.0 * nodes / (t[0] * 1e6), t[1]);
}

template <int MODE, int VEC, int PL>
float run(const double* in, double* out, int chunk, int reps) {
	dim3 grid((N / chunk) * (N / PL));
	dim3 block(512 / VEC * PL);
	hipEvent_t a, b;
	CK(hipEventCreate(&a));
	CK(hipEventCreate(&b));
	hipLaunchKernelGGL((k_probe<MODE, VEC, PL>), grid, block, 0, 0, in, out, chunk);
	CK(hipDeviceSynchronize());
	CK(hipEventRecord(a));
	for (int r = 0; r < reps; r++)
		hipLaunchKernelGGL((k_probe<MODE, VEC, PL>), grid, block, 0, 0, in, out, chunk);
	CK(hipEventRecord(b));
	CK(hipEventSynchronize(b));
	float ms = 0;
	CK(hipEventElapsedTime(&ms, a, b));
	return ms / reps;
}

template <int VEC, int PL>
void family(const double* in, double* out, int chunk) {
	const double nodes = (double)N * N * N;
	const float t0 = run<0, VEC, PL>(in, out, chunk, 10);
	const float t1 = run<1, VEC, PL>(in, out, chunk, 10);
	const float t2 = run<2, VEC, PL>(in, out, chunk, 10);
	std::printf("vec %d planes/block %d chunk %3d: copy %.3f ms (%.0f GB/s)  xpat %.3f ms (%.0f GB/s)  "
	            "xpat_ns %.3f ms\n",
	            VEC, PL, chunk, t0, 144.0 * nodes / (t0 * 1e6), t1, 144.0 * nodes / (t1 * 1e6), t2);
}

int main() {
	const size_t bytes = (size_t)9 * CS * sizeof(double);
	double *in, *out;
	CK(hipMalloc(&in, bytes));
	CK(hipMalloc(&out, bytes));
	CK(hipMemset(in, 0, bytes));
	CK(hipMemset(out, 0, bytes));
	if (std::getenv("BOX_ONLY")) {  // box characterisation: HBM copy and fp64 VALU, each alone
		int dev = 0, cus = 256;
		CK(hipGetDevice(&dev));
		CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev));
		copy_span(in, out);
		valu_span(out, cus);
		copy_span(in, out);
		valu_span(out, cus);
		return 0;
	}
	if (std::getenv("TZ_ONLY")) {  // two planes x two z groups per lane at one wave per SIMD
		copy_span(in, out);
		tz<2, 0, 512, 1, 1>(in, out, 128, 96 * 1024);   // = the shipped pattern, 1 block/CU
		tz<4, 0, 256, 1, 1>(in, out, 128, 96 * 1024);   // = TX4 half rows, 1 wave/SIMD
		tz<2, 0, 256, 2, 1>(in, out, 128, 96 * 1024);   // z and z+256 per lane, whole row, 1 wave/SIMD
		tz<2, 0, 256, 1, 2>(in, out, 128, 96 * 1024);   // z, z+1 (16-B loads), whole row, 1 wave/SIMD
		tz<2, 0, 256, 2, 1>(in, out, 512, 96 * 1024);
		tz<2, 0, 256, 1, 2>(in, out, 512, 96 * 1024);
		tz<2, 0, 512, 1, 1>(in, out, 512, 0);
		ops_tx<2, 540>(in, out, 128);
		tz<2, 540, 256, 2, 1>(in, out, 128, 96 * 1024);
		tz<2, 540, 256, 1, 2>(in, out, 128, 96 * 1024);
		tz<4, 540, 256, 1, 1>(in, out, 128, 96 * 1024);
		tz<2, 900, 512, 1, 1>(in, out, 512, 0);
		tz<2, 900, 256, 2, 1>(in, out, 512, 96 * 1024);
		tz<2, 900, 256, 1, 2>(in, out, 512, 96 * 1024);
		tz<4, 900, 256, 1, 1>(in, out, 512, 96 * 1024);
		return 0;
	}
	if (std::getenv("TX4_ONLY")) {  // four planes per thread at one wave per SIMD
		family<1, 1>(in, out, 128);
		family<2, 1>(in, out, 128);
		ops_tx<2, 0>(in, out, 128);
		ops_tx<2, 0>(in, out, 128, 96 * 1024);
		ops_tx<4, 0>(in, out, 128);
		ops_tx<4, 0>(in, out, 128, 96 * 1024);
		ops_tx<4, 0, false, 256>(in, out, 128, 96 * 1024);
		ops_tx<2, 0, false, 256>(in, out, 128, 96 * 1024);
		ops_tx<2, 540>(in, out, 128);
		ops_tx<4, 540>(in, out, 128, 96 * 1024);
		ops_tx<4, 540, false, 256>(in, out, 128, 96 * 1024);
		ops_tx<2, 0>(in, out, 512);
		ops_tx<4, 0, false, 256>(in, out, 512, 96 * 1024);
		return 0;
	}
	if (std::getenv("XM_ONLY")) {  // the x-marching family beside the copy and the 2-plane pattern
		family<1, 1>(in, out, 128);
		family_tx<2>(in, out, 128);
		xmarch<12, 64>(in, out);
		xmarch<12, 128>(in, out);
		xmarch<8, 128>(in, out);
		xmarch<4, 128>(in, out);
		return 0;
	}
	family<1, 1>(in, out, 128);
	family<2, 1>(in, out, 128);
	family<2, 2>(in, out, 128);
	family_tx<1>(in, out, 128);
	family_tx<2>(in, out, 128);
	family_tx<4>(in, out, 128);
	ops_tx<2, 180>(in, out, 128);
	ops_tx<2, 360>(in, out, 128);
	ops_tx<2, 540>(in, out, 128);
	ops_tx<2, 720>(in, out, 128);
	ops_tx<2, 540, true>(in, out, 128);
	ops_tx<2, 0, true>(in, out, 128, 96 * 1024);
	ops_tx<2, 540, true>(in, out, 128, 96 * 1024);
	ops_tx<2, 720, true>(in, out, 128, 96 * 1024);
	ops_tx<2, 0>(in, out, 128, 96 * 1024);
	ops_tx<2, 360>(in, out, 128, 96 * 1024);
	ops_tx<2, 540>(in, out, 128, 96 * 1024);
	ops_tx<2, 720>(in, out, 128, 96 * 1024);
	return 0;
}
