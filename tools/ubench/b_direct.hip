// Probe: config B decode (f32 + utf8, 1000 x 100k-row blocks, utf8 index
// stride 512) with a "direct" design -- no LDS ring, no loader wave.  Every
// wave owns virtual blocks of V rows (multiples of the index stride) and
// starts its utf8 running sum at the index entry; per 64-row chunk a lane
// loads its row's (start, end) offsets with one dwordx4, then a 24-byte window
// of the row (dwordx4 + dwordx2) into registers, and decodes from registers.
// Loads of the next chunk are issued before the current one is decoded.
// Also: a streaming ceiling probe of the same byte mix.
//   hipcc --offload-arch=gfx950 -O3 -std=c++17 b_direct.hip -o b_direct
#include <hip/hip_runtime.h>

#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#define CK(x)                                                                                  \
    do {                                                                                       \
        hipError_t e_ = (x);                                                                   \
        if (e_ != hipSuccess) {                                                                \
            std::fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            std::exit(1);                                                                      \
        }                                                                                      \
    } while (0)

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef unsigned int u32x2 __attribute__((ext_vector_type(2)));
typedef unsigned int u32x3 __attribute__((ext_vector_type(3)));
typedef uint32_t __attribute__((aligned(1))) u32u;
typedef uint16_t __attribute__((aligned(1))) u16u;
typedef uint64_t __attribute__((aligned(1))) u64u;
#define DEV __device__ __forceinline__

struct Blk {
    const uint8_t* data;
    const uint64_t* row_off;
    uint64_t n;
    uint64_t bytes;
    const uint64_t* uidx;
};
struct Out {
    uint32_t* f;
    uint64_t* vf;
    uint64_t* vs;
    int32_t* off;
    uint8_t* str;
};
struct VB {
    uint32_t b, r0, r1, pad;
};

constexpr uint32_t BS = 1, FO_F = 1, FO_S = 5, CAP = 8, FIX = 9;

DEV uint32_t lane_id() { return __builtin_amdgcn_mbcnt_hi(~0u, __builtin_amdgcn_mbcnt_lo(~0u, 0u)); }
DEV uint32_t sgpr(uint32_t v) { return __builtin_amdgcn_readfirstlane(v); }
DEV uint64_t sgpr64(uint64_t v) { return ((uint64_t)sgpr((uint32_t)(v >> 32)) << 32) | sgpr((uint32_t)v); }
DEV uint32_t wave_scan(uint32_t v) {
    v += __builtin_amdgcn_update_dpp(0u, v, 0x111, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x112, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x114, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x118, 0xF, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x142, 0xA, 0xF, false);
    v += __builtin_amdgcn_update_dpp(0u, v, 0x143, 0xC, 0xF, false);
    return v;
}
#define GAS __attribute__((address_space(1)))
template <class T> DEV GAS T* gp(T* p) { return (GAS T*)p; }
template <class T> DEV const GAS T* gp(const T* p) { return (const GAS T*)p; }
// an address the optimizer cannot turn back into a branch (a select of two
// store targets becomes two predicated stores otherwise)
template <class T> DEV GAS T* opaque(GAS T* p) {
    uint64_t a = (uint64_t)p;
    asm volatile("" : "+v"(a));
    return (GAS T*)a;
}
DEV uint32_t ab(uint32_t hi, uint32_t lo, uint32_t s) { return __builtin_amdgcn_alignbyte(hi, lo, s); }

struct Win {
    uint32_t w[6];
};
struct Q {
    uint64_t s;
    uint32_t e;
};

DEV Q ldq(const uint64_t* ro, uint64_t r) {
    const u32x4 v = *(const u32x4*)(ro + r);
    return Q{((uint64_t)v.y << 32) | v.x, v.z};
}
DEV Win ldwin(const uint8_t* a4) {
    Win W;
    const u32x4 x = *(const u32x4*)a4;
    const u32x2 y = *(const u32x2*)(a4 + 16);
    W.w[0] = x.x; W.w[1] = x.y; W.w[2] = x.z; W.w[3] = x.w; W.w[4] = y.x; W.w[5] = y.y;
    return W;
}

// slow path of one lane: exact reference semantics from global memory
// (read.rs:39-55); returns the string length (0 for a null/malformed cell),
// sets *bad for a malformed row
DEV uint32_t slow_row(const GAS uint8_t* row, uint32_t rl, bool& vf, bool& vs, uint32_t& fv, uint32_t& spay, bool& bad) {
    bad = false;
    if (rl == 0) { vf = vs = false; fv = 0; return 0; }
    if (rl < BS) { bad = true; vf = vs = false; fv = 0; return 0; }
    const uint32_t bits = row[0];
    vf = !(bits & 1);
    vs = !(bits & 2);
    fv = 0;
    if (vf) {
        if (FO_F + 4 > rl) { bad = true; vf = false; }
        else fv = *(const GAS u32u*)(row + FO_F);
    }
    uint32_t len = 0;
    if (vs) {
        if (FO_S + 4 > rl) { bad = true; vs = false; return 0; }
        const uint32_t sl = *(const GAS u32u*)(row + FO_S);
        const uint32_t vlen = rl - BS;
        if (sl > vlen - 4) { bad = true; vs = false; return 0; }
        const uint32_t l = *(const GAS u32u*)(row + BS + sl);
        if (l > vlen - 4 - sl) { bad = true; vs = false; return 0; }
        spay = BS + sl + 4;
        len = l;
    }
    return len;
}


struct Meta {
    uint64_t ra;  // row address
    uint32_t rl;  // row length (0: missing or past the virtual block)
    uint32_t safe;
};

// A chunk is "common" when every row is on the fast path and every string
// is 0 or 4..8 bytes: then its decode issues a fixed set of stores (lanes with
// nothing to write aimed at a sink), with no branch, so the compiler's vmcnt
// bookkeeping of the prefetched loads stays exact.
DEV bool common_row(const Meta& M, const Win& W) {
    const uint32_t sh = (uint32_t)M.ra & 3u;
    const uint32_t r0w = ab(W.w[1], W.w[0], sh), r1w = ab(W.w[2], W.w[1], sh), r2w = ab(W.w[3], W.w[2], sh),
                   r3w = ab(W.w[4], W.w[3], sh);
    const uint32_t rl = M.rl;
    const bool vs = rl >= FIX && !(r0w & 2);
    const uint32_t slot = ab(r2w, r1w, 1), lenw = ab(r3w, r2w, 1);
    const bool fast = M.safe && (rl == 0 || (rl >= FIX && (!vs || (slot == CAP && lenw == rl - 13 && lenw <= 8))));
    return fast && (!vs || lenw == 0 || lenw >= 4);
}

template <bool ABL_NOSTR>
DEV void decode_common(const Meta& M, const Win& W, uint32_t c0, uint32_t r1, const Out& O, uint64_t& run, uint32_t& nf,
                       uint32_t& ns, uint32_t lane, uint8_t* sink, bool live = true) {
    const uint32_t r = c0 + lane;
    const bool act = live && r < r1;
    const uint32_t rl = M.rl;
    const uint32_t sh = (uint32_t)M.ra & 3u;
    uint32_t rw[4];
#pragma unroll
    for (int j = 0; j < 4; j++) rw[j] = ab(W.w[j + 1], W.w[j], sh);
    const bool vf = rl >= FIX && !(rw[0] & 1);
    const bool vs = rl >= FIX && !(rw[0] & 2);
    const uint32_t fv = vf ? ab(rw[1], rw[0], FO_F) : 0u;
    const uint32_t lenw = ab(rw[3], rw[2], 1);  // row byte 9
    const uint32_t d0 = (sh + 13) >> 2, s0 = (sh + 13) & 3;
    const uint32_t u0 = d0 == 3 ? W.w[3] : W.w[4];
    const uint32_t u1 = d0 == 3 ? W.w[4] : W.w[5];
    const uint32_t u2 = d0 == 3 ? W.w[5] : 0u;
    GAS uint8_t* snk = gp(sink) + 8 * lane;
    const uint32_t len = vs ? lenw : 0u;
    const uint32_t incl = wave_scan(len);
    const uint32_t tot = __builtin_amdgcn_readlane(incl, 63);
    const uint64_t e = run + incl;
    *opaque(act ? (GAS int32_t*)(gp(O.off) + r + 1) : (GAS int32_t*)snk) = (int32_t)e;
    *opaque(act ? (GAS uint32_t*)(gp(O.f) + r) : (GAS uint32_t*)snk) = fv;
    const uint64_t mf = __ballot(vf), ms = __ballot(vs);
    const uint64_t am = __ballot(act);
    nf += __popcll(am & ~mf);
    ns += __popcll(am & ~ms);
    *opaque(live && lane < 2 ? gp(lane == 0 ? O.vf : O.vs) + (c0 >> 6) : (GAS uint64_t*)snk) = lane == 0 ? mf : ms;
    if (!ABL_NOSTR) {
        const bool has = len != 0;
        GAS uint8_t* vb_ = gp(O.str) + (e - len);
        const uint32_t head = ab(u1, u0, s0);
        const uint32_t x = s0 + len - 4;
        const uint32_t tail = x < 4 ? ab(u1, u0, x) : ab(u2, u1, x - 4);
        *opaque((GAS u32u*)(has ? vb_ : snk)) = head;
        *opaque((GAS u32u*)(has ? vb_ + len - 4 : snk)) = tail;
    }
    run += tot;
}

// the general path of one chunk: exact reference semantics, any row
DEV void decode_general(const uint64_t* ro, const uint8_t* base, uint64_t lim, uint32_t c0, uint32_t r1, const Out& O,
                        uint64_t& run, uint32_t& nf, uint32_t& ns, uint32_t lane, unsigned int* errflag) {
    const uint32_t r = c0 + lane;
    const bool act = r < r1;
    uint32_t rl = 0;
    uint64_t s = 0;
    if (act) {
        s = gp(ro)[r];
        rl = (uint32_t)(gp(ro)[r + 1] - s);
    }
    bool vf = false, vs = false, bad = false;
    uint32_t fv = 0, spay = 0;
    const GAS uint8_t* row = gp(base) + s;
    const uint32_t len = act ? slow_row(row, rl, vf, vs, fv, spay, bad) : 0u;
    if (bad) atomicOr(errflag, 1u);
    if (!vf) fv = 0;
    const uint32_t incl = wave_scan(len);
    const uint32_t tot = __builtin_amdgcn_readlane(incl, 63);
    const uint64_t e = run + incl;
    if (act) gp(O.off)[r + 1] = (int32_t)e;
    if (act) gp(O.f)[r] = fv;
    const uint64_t mf = __ballot(vf), ms = __ballot(vs);
    const uint64_t am = __ballot(act);
    nf += __popcll(am & ~mf);
    ns += __popcll(am & ~ms);
    if (lane < 2) gp(lane == 0 ? O.vf : O.vs)[c0 >> 6] = lane == 0 ? mf : ms;
    if (len) {
        GAS uint8_t* vb_ = gp(O.str) + (e - len);
        for (uint32_t q = 0; q < len; q++) vb_[q] = row[spay + q];
    }
    run += tot;
}

template <uint32_t WPB, uint32_t R, bool ABL_NOSTR>
__global__ void __launch_bounds__(64 * WPB) dec_direct(const Blk* __restrict__ blocks, const Out* __restrict__ outs,
                                                       const VB* __restrict__ vbs, uint32_t nvb,
                                                       unsigned long long* nulls, unsigned long long* lens,
                                                       unsigned int* errflag, uint8_t* sink) {
    const uint32_t lane = lane_id();
    const uint32_t gw = sgpr(blockIdx.x * WPB + (threadIdx.x >> 6));
    const uint32_t nw = gridDim.x * WPB;
    for (uint32_t v = gw; v < nvb; v += nw) {
        const VB vb = vbs[v];
        const uint32_t b = sgpr(vb.b), r0 = sgpr(vb.r0), r1 = sgpr(vb.r1);
        const Blk B = blocks[b];
        const Out O = outs[b];
        const uint8_t* base = (const uint8_t*)sgpr64((uint64_t)B.data);
        const uint64_t* ro = (const uint64_t*)sgpr64((uint64_t)B.row_off);
        const uint64_t n = sgpr64(B.n);
        const uint64_t lim = sgpr64(((uint64_t)B.data + B.bytes + 15) & ~15ull);
        uint64_t run = r0 ? sgpr64(B.uidx[r0 >> 9]) : 0;
        uint32_t nf = 0, ns = 0;
        // q loads: (start, end) of rows c + 64k + lane (clamped into the virtual block)
        auto ldqs = [&](uint32_t c, u32x3 (&q)[R]) {
#pragma unroll
            for (uint32_t k = 0; k < R; k++) {
                const uint32_t r = c + 64 * k + lane;
                q[k] = *(const GAS u32x3*)gp(ro + (r < r1 ? r : r1 - 1));
            }
        };
        auto metas = [&](uint32_t c, const u32x3 (&q)[R], Meta (&M)[R], Win (&W)[R]) {
#pragma unroll
            for (uint32_t k = 0; k < R; k++) {
                const uint32_t r = c + 64 * k + lane;
                const uint64_t s = ((uint64_t)q[k].y << 32) | q[k].x;
                M[k].ra = (uint64_t)base + s;
                M[k].rl = r < r1 ? q[k].z - q[k].x : 0u;
                const uint64_t a4 = M[k].ra & ~3ull;
                M[k].safe = a4 + 24 <= lim;
                const GAS uint8_t* p = gp((const uint8_t*)(M[k].safe ? a4 : (uint64_t)base));
                const u32x4 x = *(const GAS u32x4*)p;
                const u32x2 y = *(const GAS u32x2*)(p + 16);
                W[k].w[0] = x.x; W[k].w[1] = x.y; W[k].w[2] = x.z; W[k].w[3] = x.w; W[k].w[4] = y.x; W[k].w[5] = y.y;
            }
        };
        auto all_common = [&](const Meta (&M)[R], const Win (&W)[R]) {
            bool ok = true;
#pragma unroll
            for (uint32_t k = 0; k < R; k++) ok = ok && common_row(M[k], W[k]);
            return __ballot(!ok) == 0;
        };
        constexpr uint32_t STEP = 64 * R;
        // Pipelined runs of common batches (R chunks): the windows of batch
        // i+1 and the offsets of batch i+2 are in flight while batch i is
        // decoded.  A batch that is not common ends the run; its first chunk
        // goes through the general path and the next run starts after it.
        uint32_t c = r0;
        while (c < r1) {
            u32x3 qA[R], qB[R];
            Meta mA[R], mB[R];
            Win wA[R], wB[R];
            ldqs(c, qA);
            metas(c, qA, mA, wA);
            ldqs(c + STEP, qB);
            // a dead batch (every store to the sink): the loop is then entered
            // with the same memory operations in flight as on its back edge,
            // so the compiler's waits there are the steady-state counts
#pragma unroll
            for (uint32_t k = 0; k < R; k++) decode_common<ABL_NOSTR>(mA[k], wA[k], c, r1, O, run, nf, ns, lane, sink, false);
            for (;;) {
                metas(c + STEP, qB, mB, wB);
                ldqs(c + 2 * STEP, qA);
                if (!all_common(mA, wA)) break;
#pragma unroll
                for (uint32_t k = 0; k < R; k++) decode_common<ABL_NOSTR>(mA[k], wA[k], c + 64 * k, r1, O, run, nf, ns, lane, sink);
                c += STEP;
                if (c >= r1) break;
                metas(c + STEP, qA, mA, wA);
                ldqs(c + 2 * STEP, qB);
                if (!all_common(mB, wB)) break;
#pragma unroll
                for (uint32_t k = 0; k < R; k++) decode_common<ABL_NOSTR>(mB[k], wB[k], c + 64 * k, r1, O, run, nf, ns, lane, sink);
                c += STEP;
                if (c >= r1) break;
            }
            if (c < r1) {
                decode_general(ro, base, lim, c, r1, O, run, nf, ns, lane, errflag);
                c += 64;
            }
        }
        if (lane == 0) {
            if (nf) atomicAdd(nulls + 2 * b, (unsigned long long)nf);
            if (ns) atomicAdd(nulls + 2 * b + 1, (unsigned long long)ns);
            if (r1 == n) lens[b] = run;
            if (r0 == 0) O.off[0] = 0;
        }
    }
}

// streaming ceiling: each thread reads 2*U 16-B words (grid stride) and writes U
__global__ void __launch_bounds__(256) mix(const u32x4* __restrict__ in, u32x4* __restrict__ out, size_t nout) {
    constexpr int U = 4;
    const size_t nt = (size_t)gridDim.x * blockDim.x;
    for (size_t o = blockIdx.x * (size_t)blockDim.x + threadIdx.x; o < nout; o += nt * U) {
        u32x4 a[U], b[U];
#pragma unroll
        for (int k = 0; k < U; k++) {
            const size_t j = o + k * nt;
            if (j < nout) { a[k] = __builtin_nontemporal_load(in + 2 * j); b[k] = __builtin_nontemporal_load(in + 2 * j + 1); }
        }
#pragma unroll
        for (int k = 0; k < U; k++) {
            const size_t j = o + k * nt;
            if (j < nout) out[j] = a[k] ^ b[k];
        }
    }
}

static std::string istr(uint64_t i) { return std::to_string(i); }

int main(int argc, char** argv) {
    const uint32_t N = 100000, K = argc > 1 ? std::atoi(argv[1]) : 1000;
    // host block: config B rows (bitset 0xFC: both cells non-null; f32 = i; slot 8; len; bytes)
    std::vector<uint8_t> blob;
    std::vector<uint64_t> off(N + 1);
    std::vector<uint32_t> ef(N);
    std::vector<int32_t> eoff(N + 1, 0);
    std::string estr;
    for (uint32_t i = 0; i < N; i++) {
        off[i] = blob.size();
        const std::string s = istr(i);
        const float f = (float)i;
        uint32_t fb;
        std::memcpy(&fb, &f, 4);
        ef[i] = fb;
        blob.push_back(0xFC);
        for (int k = 0; k < 4; k++) blob.push_back((fb >> (8 * k)) & 0xFF);
        const uint32_t slot = CAP, len = (uint32_t)s.size();
        for (int k = 0; k < 4; k++) blob.push_back((slot >> (8 * k)) & 0xFF);
        for (int k = 0; k < 4; k++) blob.push_back((len >> (8 * k)) & 0xFF);
        blob.insert(blob.end(), s.begin(), s.end());
        estr += s;
        eoff[i + 1] = (int32_t)estr.size();
    }
    off[N] = blob.size();
    const uint32_t S = 512, nix = (N + S - 1) / S + 1;
    std::vector<uint64_t> ix(nix);
    for (uint32_t j = 0; j < nix; j++) ix[j] = (uint64_t)eoff[std::min<uint32_t>(j * S, N)];
    const uint64_t bb = blob.size();
    std::printf("block: %u rows, %llu blob bytes, %zu string bytes\n", N, (unsigned long long)bb, estr.size());

    // device: K copies
    std::vector<Blk> hb(K);
    std::vector<Out> ho(K);
    std::vector<void*> frees;
    auto dal = [&](size_t n) { void* p; CK(hipMalloc(&p, n)); frees.push_back(p); return p; };
    for (uint32_t k = 0; k < K; k++) {
        uint8_t* d = (uint8_t*)dal((bb + 15) / 16 * 16 + 16);
        uint64_t* o = (uint64_t*)dal(8 * (N + 1));
        uint64_t* u = (uint64_t*)dal(8 * nix);
        CK(hipMemcpy(d, blob.data(), bb, hipMemcpyHostToDevice));
        CK(hipMemcpy(o, off.data(), 8 * (N + 1), hipMemcpyHostToDevice));
        CK(hipMemcpy(u, ix.data(), 8 * nix, hipMemcpyHostToDevice));
        hb[k] = Blk{d, o, N, bb, u};
        const size_t bm = ((N + 7) / 8 + 7) / 8 * 8;
        ho[k] = Out{(uint32_t*)dal(4 * N), (uint64_t*)dal(bm), (uint64_t*)dal(bm), (int32_t*)dal(4 * (N + 1)),
                    (uint8_t*)dal(estr.size() + 16)};
    }
    Blk* dB = (Blk*)dal(sizeof(Blk) * K);
    Out* dO = (Out*)dal(sizeof(Out) * K);
    CK(hipMemcpy(dB, hb.data(), sizeof(Blk) * K, hipMemcpyHostToDevice));
    CK(hipMemcpy(dO, ho.data(), sizeof(Out) * K, hipMemcpyHostToDevice));
    unsigned long long* dn = (unsigned long long*)dal(16 * K);
    unsigned long long* dl = (unsigned long long*)dal(8 * K);
    unsigned int* derr = (unsigned int*)dal(4);
    uint8_t* dsink = (uint8_t*)dal(4096);

    const double in_b = (double)(bb + 8 * (N + 1) + 8 * nix) * K;
    const double out_b = (double)(4.0 * N + 4.0 * (N + 1) + estr.size()) * K;
    std::printf("algorithmic bytes per launch: %.0f (in %.0f out %.0f)\n", in_b + out_b, in_b, out_b);

    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    int cus = 0;
    CK(hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, 0));

    auto check = [&](const char* tag) {
        bool ok = true;
        for (uint32_t k : {0u, K / 2, K - 1}) {
            std::vector<uint32_t> f(N);
            std::vector<int32_t> o(N + 1);
            std::string s(estr.size(), '\0');
            unsigned long long nl[2], ln;
            CK(hipMemcpy(f.data(), ho[k].f, 4 * N, hipMemcpyDeviceToHost));
            CK(hipMemcpy(o.data(), ho[k].off, 4 * (N + 1), hipMemcpyDeviceToHost));
            CK(hipMemcpy(&s[0], ho[k].str, s.size(), hipMemcpyDeviceToHost));
            CK(hipMemcpy(nl, dn + 2 * k, 16, hipMemcpyDeviceToHost));
            CK(hipMemcpy(&ln, dl + k, 8, hipMemcpyDeviceToHost));
            if (f != ef || o != eoff || s != estr || nl[0] || nl[1] || ln != estr.size()) {
                ok = false;
                size_t bf = 0, bo = 0, bs = 0;
                while (bf < N && f[bf] == ef[bf]) bf++;
                while (bo <= N && o[bo] == eoff[bo]) bo++;
                while (bs < s.size() && s[bs] == estr[bs]) bs++;
                std::printf("  %s MISMATCH block %u: f@%zu o@%zu s@%zu nulls %llu %llu len %llu\n", tag, k, bf, bo, bs,
                            nl[0], nl[1], ln);
            }
        }
        unsigned int er = 0;
        CK(hipMemcpy(&er, derr, 4, hipMemcpyDeviceToHost));
        std::printf("  %s check %s (errflag %u)\n", tag, ok ? "OK" : "FAILED", er);
    };

    auto run_direct = [&](auto kern, uint32_t wpb, uint32_t wpc, uint32_t V, const char* tag, bool chk) {
        std::vector<VB> vbs;
        for (uint32_t k = 0; k < K; k++)
            for (uint32_t r = 0; r < N; r += V) vbs.push_back(VB{k, r, std::min(N, r + V), 0});
        VB* dv = (VB*)dal(sizeof(VB) * vbs.size());
        CK(hipMemcpy(dv, vbs.data(), sizeof(VB) * vbs.size(), hipMemcpyHostToDevice));
        const uint32_t grid = cus * wpc / wpb;
        float best = 1e9, sum = 0;
        const int reps = 12;
        for (int rep = 0; rep < reps + 3; rep++) {
            CK(hipMemsetAsync(dn, 0, 16 * K));
            CK(hipMemsetAsync(derr, 0, 4));
            CK(hipEventRecord(e0));
            hipLaunchKernelGGL(kern, dim3(grid), dim3(64 * wpb), 0, 0, dB, dO, dv, (uint32_t)vbs.size(), dn, dl, derr, dsink);
            CK(hipEventRecord(e1));
            CK(hipEventSynchronize(e1));
            float ms;
            CK(hipEventElapsedTime(&ms, e0, e1));
            if (rep >= 3) { best = std::min(best, ms); sum += ms; }
        }
        std::printf("%-28s wpb %u waves/CU %2u V %5u: best %.4f ms avg %.4f ms = %.0f GB/s (frac %.3f avg)\n", tag, wpb,
                    wpc, V, best, sum / reps, (in_b + out_b) / (sum / reps) / 1e6, (in_b + out_b) / (sum / reps) / 8e9);
        if (chk) check(tag);
    };

    run_direct(dec_direct<4, 1, false>, 4, 16, 1024, "direct R1", true);
    run_direct(dec_direct<4, 2, false>, 4, 16, 1024, "direct R2", true);
    run_direct(dec_direct<4, 4, false>, 4, 16, 1024, "direct R4", true);
    for (uint32_t wpc : {8u, 16u, 24u, 32u})
        for (uint32_t V : {512u, 1024u, 2048u}) {
            run_direct(dec_direct<4, 1, false>, 4, wpc, V, "direct R1", false);
            run_direct(dec_direct<4, 2, false>, 4, wpc, V, "direct R2", false);
        }
    run_direct(dec_direct<4, 4, false>, 4, 16, 2048, "direct R4", false);
    run_direct(dec_direct<4, 4, false>, 4, 8, 2048, "direct R4", false);
    run_direct(dec_direct<8, 2, false>, 8, 32, 1024, "direct wpb8 R2", true);
    run_direct(dec_direct<4, 2, true>, 4, 16, 1024, "direct R2 NOSTR", false);
    run_direct(dec_direct<4, 2, true>, 4, 32, 1024, "direct R2 NOSTR", false);

    // ceiling probe with the same mix (in bytes read, out bytes written)
    {
        const size_t nout = (size_t)(out_b / 16), nin = 2 * nout;
        u32x4* pin = (u32x4*)dal(16 * nin);
        u32x4* pout = (u32x4*)dal(16 * nout);
        CK(hipMemset(pin, 1, 16 * nin));
        for (uint32_t g : {1024u, 2048u, 4096u, 8192u}) {
            float best = 1e9, sum = 0;
            for (int rep = 0; rep < 13; rep++) {
                CK(hipEventRecord(e0));
                hipLaunchKernelGGL(mix, dim3(g), dim3(256), 0, 0, pin, pout, nout);
                CK(hipEventRecord(e1));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (rep >= 3) { best = std::min(best, ms); sum += ms; }
            }
            const double by = 16.0 * nin + 16.0 * nout;
            std::printf("mix ceiling grid %5u: read %.2f GB write %.2f GB best %.4f avg %.4f ms = %.0f GB/s (frac %.3f)\n", g,
                        16.0 * nin / 1e9, 16.0 * nout / 1e9, best, sum / 10, by / (sum / 10) / 1e6, by / (sum / 10) / 8e9);
        }
    }
    for (void* p : frees) (void)hipFree(p);
    return 0;
}
