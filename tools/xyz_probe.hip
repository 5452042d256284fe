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
