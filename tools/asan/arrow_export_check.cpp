// Host-only check of the library's host code under AddressSanitizer /
// UndefinedBehaviorSanitizer (no GPU): murr_arrow_export with every dtype,
// with and without nulls, empty and zero-column batches, a mixed-length
// rejection (every exported byte read back, the export released); and the
// Arrow IPC framing of murr_ipc.cpp (schema and record-batch messages at
// several alignments, the size query, a short buffer).
//   hipcc -O1 -g -std=c++17 -Xarch_host -fsanitize=address -Xarch_host -fsanitize=undefined \
//     -Iinclude -Imurr_amd/csrc tools/asan/arrow_export_check.cpp murr_amd/csrc/murr_arrow.cpp \
//     murr_amd/csrc/murr_ipc.cpp -o /tmp/arrow_export_check
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "murr_codec.h"

static int fails = 0;
#define CHECK(c)                                                        \
    do {                                                                \
        if (!(c)) {                                                     \
            std::fprintf(stderr, "%s:%d CHECK %s\n", __FILE__, __LINE__, #c); \
            fails++;                                                    \
        }                                                               \
    } while (0)

int main() {
    const uint64_t n = 1000;
    std::vector<uint8_t> validity((n + 7) / 8, 0xFF);
    validity[3] = 0xF0;
    std::vector<int64_t> i64(n);
    for (uint64_t i = 0; i < n; i++) i64[i] = (int64_t)i * 7;
    std::vector<uint8_t> bools((n + 7) / 8, 0xA5);
    std::vector<int32_t> offs(n + 1);
    std::string bytes;
    for (uint64_t i = 0; i < n; i++) {
        offs[i] = (int32_t)bytes.size();
        bytes += std::string(i % 13, 'a' + (char)(i % 26));
    }
    offs[n] = (int32_t)bytes.size();
    const uint32_t dts[] = {MURR_INT64, MURR_BOOL, MURR_UTF8, MURR_FLOAT64, MURR_UINT8};
    for (int variant = 0; variant < 3; variant++) {
        const uint64_t len = variant == 2 ? 0 : n;
        std::vector<murr_host_array_t> a(5);
        for (int k = 0; k < 5; k++) {
            murr_host_array_t& h = a[k];
            std::memset(&h, 0, sizeof h);
            h.dtype = dts[k];
            h.length = len;
            h.null_count = variant == 1 ? 4 : 0;
            h.validity = variant == 1 ? validity.data() : nullptr;
            if (h.dtype == MURR_UTF8) {
                h.values = (const uint8_t*)bytes.data();
                h.offsets = offs.data();
                h.values_len = len ? bytes.size() : 0;
            } else if (h.dtype == MURR_BOOL) {
                h.values = bools.data();
                h.values_len = (len + 7) / 8;
            } else {
                h.values = (const uint8_t*)i64.data();
                h.values_len = len * (h.dtype == MURR_UINT8 ? 1 : 8);
            }
        }
        const char* names[] = {"a", "b", "c", "d", "e"};
        ArrowArray arr;
        ArrowSchema sch;
        CHECK(murr_arrow_export(a.data(), 5, names, &arr, &sch) == MURR_OK);
        CHECK(arr.n_children == 5 && sch.n_children == 5 && std::strcmp(sch.format, "+s") == 0);
        for (int k = 0; k < 5; k++) {
            const ArrowArray* c = arr.children[k];
            CHECK(c->length == (int64_t)len);
            for (int64_t b = 0; b < c->n_buffers; b++) {
                const uint8_t* p = (const uint8_t*)c->buffers[b];
                if (!p) continue;
                uint64_t nb = b == 0 ? (len + 7) / 8 : (b == 1 && dts[k] == MURR_UTF8) ? 4 * (len + 1) : a[k].values_len;
                volatile uint64_t s = 0;
                for (uint64_t j = 0; j < nb; j++) s += p[j];  // (ASan: every byte in bounds)
                if (b == 1 && dts[k] == MURR_INT64 && len) CHECK(((const int64_t*)p)[999] == 999 * 7);
            }
        }
        arr.release(&arr);
        sch.release(&sch);
        CHECK(arr.release == nullptr && sch.release == nullptr);
    }
    {  // lengths differ: rejected, nothing allocated
        murr_host_array_t a[2];
        std::memset(a, 0, sizeof a);
        a[0].dtype = a[1].dtype = MURR_INT64;
        a[0].length = 3, a[1].length = 4;
        a[0].values = a[1].values = (const uint8_t*)i64.data();
        a[0].values_len = 24, a[1].values_len = 32;
        const char* names[] = {"x", "y"};
        ArrowArray arr;
        ArrowSchema sch;
        CHECK(murr_arrow_export(a, 2, names, &arr, &sch) == MURR_E_ARGUMENT);
    }
    {  // no schema side (a caller that keeps an earlier export's schema)
        murr_host_array_t a;
        std::memset(&a, 0, sizeof a);
        a.dtype = MURR_INT64;
        a.length = 10;
        a.values = (const uint8_t*)i64.data();
        a.values_len = 80;
        const char* names[] = {"x"};
        ArrowArray arr;
        CHECK(murr_arrow_export(&a, 1, names, &arr, nullptr) == MURR_OK);
        CHECK(arr.n_children == 1 && ((const int64_t*)arr.children[0]->buffers[1])[9] == 63);
        arr.release(&arr);
    }
    {  // no columns
        ArrowArray arr;
        ArrowSchema sch;
        CHECK(murr_arrow_export(nullptr, 0, nullptr, &arr, &sch) == MURR_OK);
        arr.release(&arr);
        sch.release(&sch);
    }
    {  // IPC framing of the same arrays (host): schema + record batch
        murr_column_t cols[5];
        uint32_t off = 0;
        for (uint32_t k = 0; k < 5; k++) {
            const uint32_t sz = dts[k] == MURR_UTF8 ? 4 : dts[k] == MURR_UINT8 || dts[k] == MURR_BOOL ? 1 : 8;
            cols[k] = murr_column_t{k, dts[k], off, sz};
            off += sz;
        }
        murr_segment_t seg{5, 1, off, 0, cols};
        const uint32_t proj[] = {2, 0, 1, 4, 3, 2};
        const char* names[] = {"c", "a", "b", "e", "d", "c2"};
        std::vector<murr_host_array_t> a(6);
        for (int p = 0; p < 6; p++) {
            murr_host_array_t& h = a[p];
            std::memset(&h, 0, sizeof h);
            const uint32_t dt = dts[proj[p]];
            h.dtype = dt;
            h.length = n;
            h.null_count = p % 2 ? 4 : 0;
            h.validity = p % 2 ? validity.data() : nullptr;
            if (dt == MURR_UTF8) h.values = (const uint8_t*)bytes.data(), h.offsets = offs.data(), h.values_len = bytes.size();
            else if (dt == MURR_BOOL) h.values = bools.data(), h.values_len = (n + 7) / 8;
            else h.values = (const uint8_t*)i64.data(), h.values_len = n * (dt == MURR_UINT8 ? 1 : 8);
        }
        for (uint32_t align : {8u, 64u, 4096u}) {
            uint64_t len = 0;
            CHECK(murr_ipc_schema(&seg, proj, 6, names, align, nullptr, 0, &len) == MURR_OK && len > 0);
            std::vector<uint8_t> sm(len);
            CHECK(murr_ipc_schema(&seg, proj, 6, names, align, sm.data(), len, &len) == MURR_OK);
            CHECK(murr_ipc_batch_host(&seg, proj, 6, a.data(), n, align, nullptr, 0, &len) == MURR_OK && len > 0);
            std::vector<uint8_t> bm(len);
            CHECK(murr_ipc_batch_host(&seg, proj, 6, a.data(), n, align, bm.data(), len, &len) == MURR_OK);
            CHECK(*(const uint32_t*)bm.data() == 0xFFFFFFFFu);
            uint64_t need = 0;
            CHECK(murr_ipc_batch_host(&seg, proj, 6, a.data(), n, align, bm.data(), len - 1, &need) == MURR_E_CAPACITY);
        }
        uint8_t eos[8];
        CHECK(murr_ipc_eos(eos) == 8);
    }
    std::printf("arrow_export_check: %s\n", fails ? "FAILED" : "ok");
    return fails ? 1 : 0;
}
