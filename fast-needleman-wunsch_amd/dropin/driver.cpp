// driver.cpp -- process entry for the MI355X fill, with the CLI and stdout of the
// reference driver (src/common/driver.cpp:1-40):
//   prog <argv1.bdna> <argv2.bdna>
//   argv1 = s1 "across the top", argv2 = s2 "down the side"
//   stdout: "<fill ms>\nScore: <t[size-1]>\n"
// Timing covers only the needlemanWunsch() call (driver.cpp:26-30); the table is
// allocated and page-touched before it (driver.cpp:22-23).
#include <chrono>
#include <iostream>

#include "nw_dropin.hpp"

int main(int argc, char **argv) {
    if (argc != 3) {
        std::cout << "error: incorrect number of arguments (expected 2, got " << argc << ")"
                  << std::endl;
        return 1;
    }
    dnaArray s1, s2;
    try {
        s1 = readSequence(argv[1]);
        s2 = readSequence(argv[2]);
    } catch (std::string e) {
        std::cout << "ERROR: no such file " << e << std::endl;
        return 1;
    }
    long int size = (long int)(s1.size + 1) * (long int)(s2.size + 1);
    int *table = new int[size];
    for (long int i = 0; i < size; i += 1024) table[i] = 0;

    auto wallStart = std::chrono::system_clock::now();
    needlemanWunsch(s1, s2, table);
    auto wallDiff = std::chrono::system_clock::now() - wallStart;

    int wallMsec = std::chrono::duration_cast<std::chrono::milliseconds>(wallDiff).count();
    std::cout << wallMsec;
    std::cout << "\nScore: " << table[size - 1] << std::endl;
    delete[] table;
    delete[] s1.dna;
    delete[] s2.dna;
    return 0;
}
