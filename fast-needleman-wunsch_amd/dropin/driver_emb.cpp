// driver_emb.cpp -- process entry with the CLI of the reference's second driver
// (src/common/driver2.cpp:1-44), the caller of the emb-layout fills:
//   prog <argv1.bdna> <argv2.bdna>        (argv1 across the top, argv2 down the side)
//   table: (s1.size + 2) x (s2.size + 1) ints, one leading progress column
//   stdout: the fill's wall milliseconds only, no newline and no score
// Argument and file errors print the same messages as driver.cpp and return 1.
#include <chrono>
#include <iostream>

#include "nw_dropin.hpp"

int main(int argc, char **argv) {
    if (argc != 3) {
        std::cout << "error: incorrect number of arguments (expected 2, got " << argc << ")"
                  << std::endl;
        return 1;
    }
    dnaArray top, side;
    try {
        top = readSequence(argv[1]);
        side = readSequence(argv[2]);
    } catch (std::string missing) {
        std::cout << "ERROR: no such file " << missing << std::endl;
        return 1;
    }
    const unsigned long long cells = (unsigned long long)(top.size + 2) * (unsigned long long)(side.size + 1);
    int *emb = new int[cells];

    const auto t0 = std::chrono::system_clock::now();
    needlemanWunsch(top, side, emb);
    const auto elapsed = std::chrono::system_clock::now() - t0;
    std::cout << std::chrono::duration_cast<std::chrono::milliseconds>(elapsed).count();

    delete[] emb;
    delete[] top.dna;
    delete[] side.dna;
    return 0;
}
