// ref_plugin_decl.hpp -- TEST INFRASTRUCTURE.  The declaration a reference fill TU
// provides to src/common/driver.cpp by textual order (serial.cpp:4 defines
// needlemanWunsch above `#include "driver.cpp"`, serial.cpp:38-39).  Force-included
// when the reference's unmodified driver.cpp is compiled on its own and linked
// against the MI355X drop-in TU (oracle/Makefile, target ref-dropin).
#pragma once
void needlemanWunsch(dnaArray s1, dnaArray s2, int *t);
