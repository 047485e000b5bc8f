// CPU check of the host packer (host_pack.cpp) for tests/test_pack_records.py: packs a window
// set given in a binary file with and without inline N records (nrec.h) and writes the images
// back, plus span_scan() on the lengths.
//   pack_records <in.bin> <out.bin>
// in.bin:  u32 n, u32 len[n], then each window's Dna5 bytes back to back
// out.bin: u32 flags_plain, u32 flags_rec, u64 span, u32 first, u32 diff, u64 n_bases,
//          codes_plain[n_bases / 16], nmask_plain[n_bases / 32], codes_rec[...], nmask_rec[...]
// (records are only valid for equal windows; the test sends equal ones for that part)
#include <cstdio>
#include <cstdlib>
#include <vector>

#include "host_pack.h"

int main(int argc, char** argv) {
    if (argc != 3) return 2;
    FILE* f = std::fopen(argv[1], "rb");
    if (!f) return 3;
    uint32_t n = 0;
    if (std::fread(&n, 4, 1, f) != 1) return 4;
    std::vector<uint32_t> len(n);
    if (n && std::fread(len.data(), 4, n, f) != n) return 5;
    std::vector<uint64_t> off(n);
    uint64_t total = 0;
    for (uint32_t i = 0; i < n; ++i) {
        off[i] = total;
        total += len[i];
    }
    std::vector<uint8_t> bases(total + 64);
    if (total && std::fread(bases.data(), 1, total, f) != total) return 6;
    std::fclose(f);
    uint32_t first = 0, diff = 0;
    const uint64_t span = acamd::span_scan(len.data(), n, &first, &diff);
    uint64_t nb = 0;
    for (uint32_t i = 0; i < n; ++i) nb += acamd::image_span(len[i]);
    nb = nb ? nb : 32;
    std::vector<uint32_t> c0(nb / 16, 0xdeadbeefu), m0(nb / 32, 0xdeadbeefu), c1(nb / 16, 0), m1(nb / 32, 0);
    std::vector<uint64_t> st(n);
    std::vector<uint32_t> ln(n);
    // (the packer writes every code word of a window's slot; nmask words only where it is told to)
    const uint32_t fp = acamd::pack_dna5_range(bases.data(), off.data(), len.data(), 0, n, 0, c0.data(), m0.data(),
                                               st.data(), ln.data(), false);
    const uint32_t fr = acamd::pack_dna5_range(bases.data(), off.data(), len.data(), 0, n, 0, c1.data(), m1.data(),
                                               st.data(), ln.data(), true);
    FILE* o = std::fopen(argv[2], "wb");
    if (!o) return 7;
    std::fwrite(&fp, 4, 1, o);
    std::fwrite(&fr, 4, 1, o);
    std::fwrite(&span, 8, 1, o);
    std::fwrite(&first, 4, 1, o);
    std::fwrite(&diff, 4, 1, o);
    std::fwrite(&nb, 8, 1, o);
    std::fwrite(c0.data(), 4, c0.size(), o);
    std::fwrite(m0.data(), 4, m0.size(), o);
    std::fwrite(c1.data(), 4, c1.size(), o);
    std::fwrite(m1.data(), 4, m1.size(), o);
    std::fclose(o);
    return 0;
}
