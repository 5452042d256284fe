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
template <int TX, bool STORE, int KOPS = 0, bool BAR = false>
__global__ __launch_bounds__(512, 2) void k_probe_tx(const double* __restrict__ in,
                                                     double* __restrict__ out, int chunk) {
	extern __shared__ double dyn_lds[];
	__shared__ double zl[BAR ? TX : 1][6][BAR ? 516 : 1];
	const int z = threadIdx.x;
	if (z == 1023) dyn_lds[0] = 0.0;  // never true: keeps the dynamic LDS request
	const int T_ = gridDim.x, b = blockIdx.x;
	const int p = (T_ % 8 == 0) ? (b % 8) * (T_ / 8) + b / 8 : b;
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

template <int TX, int KOPS, bool BAR = false>
void ops_tx(const double* in, double* out, int chunk, size_t shm = 0) {
	const double nodes = (double)N * N * N;
	dim3 grid((N / chunk) * (N / TX));
	hipEvent_t a, b;
	CK(hipEventCreate(&a));
	CK(hipEventCreate(&b));
	for (int r = 0; r < 11; r++) {
		if (r == 1) CK(hipEventRecord(a));
		hipLaunchKernelGGL((k_probe_tx<TX, true, KOPS, BAR>), grid, dim3(512), shm, 0, in, out, chunk);
	}
	CK(hipEventRecord(b));
	CK(hipEventSynchronize(b));
	float ms = 0;
	CK(hipEventElapsedTime(&ms, a, b));
	ms /= 10;
	std::printf("TX %d planes/thread chunk %3d + %d fp64 ops/node%s%s: %.3f ms (%.0f GB/s)\n", TX, chunk, KOPS,
	            BAR ? " + Z exchange (2 barriers/row)" : "", shm ? " (1 block/CU)" : "", ms,
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
