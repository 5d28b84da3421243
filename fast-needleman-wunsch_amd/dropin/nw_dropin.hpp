// nw_dropin.hpp -- the reference's plugin ABI for the fill, restated.
//
// The reference passes sequences as `struct dnaArray { int size; int8_t* dna; }`
// by value (src/common/helper.hpp:9-12) and selects a fill at link time through
// the symbol `void needlemanWunsch(dnaArray, dnaArray, int*)`
// (mangled _Z15needlemanWunsch8dnaArrayS_Pi; serial.cpp:4, sentinel-mt.cpp:4,
// idxarray-mt.cpp:4).  This header declares the same layout and signature so the
// MI355X TU below links in their place.
#ifndef NW_DROPIN_HPP
#define NW_DROPIN_HPP

#include <cstdint>
#include <string>

struct dnaArray {
    int size;     // offset 0
    int8_t *dna;  // offset 8
};
static_assert(sizeof(dnaArray) == 16, "dnaArray must match the reference ABI (helper.hpp:9-12)");

// Scoring constants: compile-time, like needleman-wunsch.hpp:11-13; override with
// -DNW_MATCH=.. -DNW_MISMATCH=.. -DNW_GAP=.. to build other schemes.
#ifndef NW_MATCH
#define NW_MATCH 1
#endif
#ifndef NW_MISMATCH
#define NW_MISMATCH 0
#endif
#ifndef NW_GAP
#define NW_GAP -1
#endif

// The plugin entry point (fills every cell of t, reference layout).
void needlemanWunsch(dnaArray s1, dnaArray s2, int *t);

// readSequence semantics (helper.cpp:3-25): throws std::string(fileName) when
// the file cannot be opened.
dnaArray readSequence(std::string fileName);

#endif
