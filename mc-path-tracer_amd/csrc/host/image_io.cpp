// image_io.cpp -- film output: PNG and PFM writers.
//
// The reference saves the displayed frame with stb_image_write
// (RenderingContext.cpp:114-118: stbi_write_png of the 8-bit RGB framebuffer
// that draw_to_surface filled, wavefront_kernels.cu:6-40).  Here:
//   mcpt_image_write_png  8-bit RGB PNG from an RGBA8 buffer (alpha dropped), row 0
//                         = top of the image; zlib stream of stored (uncompressed)
//                         deflate blocks, so no compression library is needed;
//   mcpt_image_write_pfm  32-bit float RGB PFM ("PF", little-endian scale -1,
//                         rows bottom-to-top per the format);
//   mcpt_film_write_png / _pfm: the context's film (tonemapped with exposure /
//                         averaged radiance Ld / samples, 0 where samples == 0).
#include <stdint.h>
#include <stdio.h>
#include <string.h>

#include <string>
#include <vector>

#include "mcpt.h"

namespace {

uint32_t crc_table[256];
bool crc_ready = false;
void crc_init() {
    for (uint32_t n = 0; n < 256; n++) {
        uint32_t c = n;
        for (int k = 0; k < 8; k++) c = (c & 1) ? 0xEDB88320u ^ (c >> 1) : c >> 1;
        crc_table[n] = c;
    }
    crc_ready = true;
}
uint32_t crc32(const uint8_t* p, size_t n, uint32_t c = 0xFFFFFFFFu) {
    if (!crc_ready) crc_init();
    for (size_t i = 0; i < n; i++) c = crc_table[(c ^ p[i]) & 0xFF] ^ (c >> 8);
    return c;
}
void be32(std::vector<uint8_t>& v, uint32_t x) {
    v.push_back((uint8_t)(x >> 24)); v.push_back((uint8_t)(x >> 16));
    v.push_back((uint8_t)(x >> 8)); v.push_back((uint8_t)x);
}
void chunk(std::vector<uint8_t>& out, const char* type, const std::vector<uint8_t>& data) {
    be32(out, (uint32_t)data.size());
    std::vector<uint8_t> td(type, type + 4);
    td.insert(td.end(), data.begin(), data.end());
    out.insert(out.end(), td.begin(), td.end());
    be32(out, crc32(td.data(), td.size()) ^ 0xFFFFFFFFu);
}

}  // namespace

extern "C" {

int mcpt_image_write_png(const char* path, uint32_t w, uint32_t h, const uint8_t* rgba) {
    if (!path || !rgba || w == 0 || h == 0) return MCPT_E_INVALID;
    // raw scanlines: filter byte 0 + RGB
    const size_t row = (size_t)w * 3 + 1;
    std::vector<uint8_t> raw(row * h);
    for (uint32_t y = 0; y < h; y++) {
        uint8_t* r = &raw[y * row];
        r[0] = 0;
        for (uint32_t x = 0; x < w; x++) {
            const uint8_t* p = rgba + ((size_t)y * w + x) * 4;
            r[1 + 3 * x] = p[0]; r[2 + 3 * x] = p[1]; r[3 + 3 * x] = p[2];
        }
    }
    // zlib: CMF/FLG, stored deflate blocks (<= 65535 bytes), adler32
    std::vector<uint8_t> z = {0x78, 0x01};
    size_t pos = 0;
    do {
        const size_t n = std::min<size_t>(65535, raw.size() - pos);
        const bool last = pos + n == raw.size();
        z.push_back(last ? 1 : 0);
        z.push_back((uint8_t)n); z.push_back((uint8_t)(n >> 8));
        z.push_back((uint8_t)~n); z.push_back((uint8_t)(~n >> 8));
        z.insert(z.end(), raw.begin() + pos, raw.begin() + pos + n);
        pos += n;
    } while (pos < raw.size());
    uint32_t a = 1, b = 0;
    for (uint8_t c : raw) { a = (a + c) % 65521u; b = (b + a) % 65521u; }
    be32(z, (b << 16) | a);
    std::vector<uint8_t> out = {0x89, 'P', 'N', 'G', 0x0D, 0x0A, 0x1A, 0x0A};
    std::vector<uint8_t> ihdr;
    be32(ihdr, w); be32(ihdr, h);
    ihdr.insert(ihdr.end(), {8, 2, 0, 0, 0});  // 8-bit, RGB, deflate, adaptive filter, no interlace
    chunk(out, "IHDR", ihdr);
    chunk(out, "IDAT", z);
    chunk(out, "IEND", {});
    FILE* f = fopen(path, "wb");
    if (!f) return MCPT_E_IO;
    const size_t wr = fwrite(out.data(), 1, out.size(), f);
    const int cl = fclose(f);
    return (wr == out.size() && cl == 0) ? MCPT_OK : MCPT_E_IO;
}

int mcpt_image_write_pfm(const char* path, uint32_t w, uint32_t h, const float* rgb) {
    if (!path || !rgb || w == 0 || h == 0) return MCPT_E_INVALID;
    FILE* f = fopen(path, "wb");
    if (!f) return MCPT_E_IO;
    bool ok = fprintf(f, "PF\n%u %u\n-1.0\n", w, h) > 0;
    for (uint32_t y = h; ok && y-- > 0;)  // PFM rows run bottom to top
        ok = fwrite(rgb + (size_t)y * w * 3, sizeof(float), (size_t)w * 3, f) == (size_t)w * 3;
    ok = (fclose(f) == 0) && ok;
    return ok ? MCPT_OK : MCPT_E_IO;
}

int mcpt_film_write_png(mcpt_ctx* ctx, float exposure, const char* path) {
    uint32_t w = 0, h = 0;
    int rc = mcpt_film_size(ctx, &w, &h);
    if (rc) return rc;
    std::vector<uint8_t> px((size_t)w * h * 4);
    if ((rc = mcpt_film_tonemap_rgba8(ctx, exposure, px.data()))) return rc;
    return mcpt_image_write_png(path, w, h, px.data());
}

int mcpt_film_write_pfm(mcpt_ctx* ctx, const char* path) {
    uint32_t w = 0, h = 0;
    int rc = mcpt_film_size(ctx, &w, &h);
    if (rc) return rc;
    std::vector<float> L((size_t)w * h * 3);
    std::vector<uint32_t> s((size_t)w * h);
    if ((rc = mcpt_film_read(ctx, L.data(), s.data()))) return rc;
    for (size_t i = 0; i < s.size(); i++)
        for (int k = 0; k < 3; k++) L[3 * i + k] = s[i] ? L[3 * i + k] / (float)s[i] : 0.f;
    return mcpt_image_write_pfm(path, w, h, L.data());
}

}  // extern "C"
