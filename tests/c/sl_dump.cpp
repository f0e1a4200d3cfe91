// Test tool (CPU): run the straight-line code generator of the library
// (uplink_amd/csrc/rs_sl_codegen.cpp) on a matrix and print what it made, for
// tests/test_sl_codegen.py, which disassembles the code with the LLVM
// disassembler and runs it in a CPU emulation against GF(2^8) arithmetic.
//   argv[1] (optional): code space in words (default: the largest region)
//   stdin:  rows nin, then rows*nin coefficient bytes (decimal), row-major
//   stdout: "split nw npass nchunks", "offsets" + one byte offset per
//           [pass][chunk][group] (-1: none), "words N" + N code words (hex)
#include <stdio.h>
#include <stdlib.h>

#include <vector>

#include "rs_sl.hpp"

int main(int argc, char **argv) {
    int rows = 0, nin = 0;
    if (scanf("%d %d", &rows, &nin) != 2 || rows < 1 || nin < 1) return 2;
    std::vector<uint8_t> M((size_t)rows * nin);
    for (auto &b : M) {
        int v;
        if (scanf("%d", &v) != 1) return 2;
        b = (uint8_t)v;
    }
    const uplink_ec::sl::Split sp = uplink_ec::sl::split_for(rows);
    const int nchunks = (nin + 2 * sp.nw - 1) / (2 * sp.nw);
    const size_t cap = argc > 1 ? (size_t)atol(argv[1]) : (size_t)uplink_ec::sl::kRegionWords;
    std::vector<uint32_t> code(cap, 0xbf810000u);
    std::vector<uint32_t> offs;
    const size_t n = uplink_ec::sl::generate(M.data(), rows, nin, code.data(), cap, offs);
    printf("split %d %d %d\n", sp.nw, sp.npass, nchunks);
    printf("offsets");
    for (uint32_t o : offs) printf(" %lld", o == uplink_ec::sl::kNoSegment ? -1LL : (long long)o);
    printf("\nwords %zu\n", n);
    for (size_t i = 0; i < n; i++) printf("%08x\n", code[i]);
    return 0;
}
