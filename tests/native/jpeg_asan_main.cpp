// Host-only driver of csrc/host/jpeg.cpp for the AddressSanitizer test (tests/test_jpeg.py): decodes
// every file named on the command line; prints "ok h w c" or "error <message>" per file.
#include <cstdio>
#include <fstream>
#include <iterator>
#include <stdexcept>
#include <vector>

#include "jpeg.hpp"

int main(int argc, char** argv) {
    for (int i = 1; i < argc; ++i) {
        std::ifstream f(argv[i], std::ios::binary);
        std::vector<uint8_t> d((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
        try {
            const cad::jpeg::Decoded o = cad::jpeg::decode(d.data(), d.size());
            std::printf("ok %d %d %d\n", o.h, o.w, o.c);
        } catch (const std::exception& e) {
            std::printf("error %s\n", e.what());
        }
    }
    return 0;
}
