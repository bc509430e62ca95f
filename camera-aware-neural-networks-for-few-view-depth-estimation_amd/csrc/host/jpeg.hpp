// Sequential-Huffman JPEG decoder reproducing libjpeg-turbo's default decompression (jpeg.cpp).
#pragma once
#include <cstddef>
#include <cstdint>
#include <vector>

namespace cad {
namespace jpeg {

struct Decoded {
    int h = 0, w = 0, c = 0;       // c: 1 (gray) or 3 (RGB)
    std::vector<uint8_t> px;       // h * w * c, row-major
};

// decode a whole JPEG file held in memory; throws std::runtime_error with a message on failure
Decoded decode(const uint8_t* data, size_t size);

}  // namespace jpeg
}  // namespace cad
