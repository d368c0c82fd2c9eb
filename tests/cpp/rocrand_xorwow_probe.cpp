// Independent pin of the XORWOW skip-ahead (tests/test_rocrand_pin.py): rocRAND's host-callable
// XORWOW engine (/opt/rocm/include/rocrand/rocrand_xorwow.h, its own 2^67-subsequence jump tables)
// applied to a given starting state.
//
//   rocrand_xorwow_probe <k> <subsequence> <d> <v0> <v1> <v2> <v3> <v4>
//
// Sets the engine's state to (d, v0..v4) -- the oracle's curand_init(seed, 0, 0) state, so rocRAND's
// own seed scramble (different constants from cuRAND's) is bypassed -- advances it by
// `subsequence` x 2^67 draws with rocRAND's discard_subsequence, then prints the state (d v0..v4)
// and k draws of rocrand(), one per line.  Host code only: no GPU is touched.
#include <cstdio>
#include <cstdlib>

#include <rocrand/rocrand_xorwow.h>

namespace {
struct Probe : rocrand_device::xorwow_engine {
    void set(const unsigned s[6]) {
        m_state.d = s[0];
        for (int i = 0; i < 5; i++) m_state.x[i] = s[1 + i];
    }
    void get(unsigned s[6]) const {
        s[0] = m_state.d;
        for (int i = 0; i < 5; i++) s[1 + i] = m_state.x[i];
    }
};
}  // namespace

int main(int argc, char** argv) {
    if (argc != 9) {
        std::fprintf(stderr, "usage: %s k subsequence d v0 v1 v2 v3 v4\n", argv[0]);
        return 2;
    }
    const int k = std::atoi(argv[1]);
    const unsigned long long sub = std::strtoull(argv[2], nullptr, 10);
    unsigned s[6];
    for (int i = 0; i < 6; i++) s[i] = (unsigned)std::strtoul(argv[3 + i], nullptr, 10);
    Probe p;
    p.set(s);
    p.discard_subsequence(sub);
    p.get(s);
    std::printf("%u %u %u %u %u %u\n", s[0], s[1], s[2], s[3], s[4], s[5]);
    for (int i = 0; i < k; i++) std::printf("%u\n", p.next());
    return 0;
}
