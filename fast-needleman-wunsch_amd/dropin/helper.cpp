// helper.cpp -- sequence input with the reference's readSequence semantics
// (src/common/helper.cpp:3-25): every byte of the file, unvalidated, as int8;
// throws std::string(fileName) when the file cannot be opened (helper.cpp:5).
#include <cstring>

#include "nw_dropin.hpp"
#include "nw_hip.h"

dnaArray readSequence(std::string fileName) {
    int8_t *buf = nullptr;
    int64_t n = 0;
    if (nw_read_bdna(fileName.c_str(), &buf, &n) != NW_OK) throw fileName;
    dnaArray ret;
    ret.size = (int)n;
    ret.dna = new int8_t[n > 0 ? n : 1];
    if (n > 0) std::memcpy(ret.dna, buf, (size_t)n);
    nw_free(buf);
    return ret;
}
