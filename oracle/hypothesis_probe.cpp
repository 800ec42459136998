// TEST INFRASTRUCTURE ONLY. The reference's own statistical test procedures: compiled by oracle/build_ref.sh against
// /root/reference/ext/hypothesis/hypothesis.h (header-only, with its cephes.h), unmodified -- the Student's t-test and
// the chi^2 test that the reference's ttest.cpp / chi2test.cpp call on their estimates (src/utils/ttest.cpp:191-240,
// chi2test.cpp). tests/test_oracle_kat.py feeds it the oracle's estimates (the reference's StudentsTTest /
// ChiSquareTest scene procedures restated over the oracle's sampler) and takes the reference's own verdict.
//
// usage: hypothesis_probe IN OUT, IN = one request per line:
//   t MEAN VARIANCE REFERENCE SAMPLES ALPHA NUM_TESTS
//   chi2 FILE N_CELLS SAMPLES MIN_EXP ALPHA NUM_TESTS   (FILE: n_cells observed then n_cells expected doubles)
// OUT = one line per request: "1" or "0" (accepted / rejected)
#include <hypothesis.h>

#include <fstream>
#include <sstream>
#include <string>
#include <vector>

int main(int argc, char **argv) {
    if (argc != 3) return 2;
    std::ifstream in(argv[1]);
    std::ofstream out(argv[2]);
    if (!in || !out) return 2;
    std::string line;
    while (std::getline(in, line)) {
        std::istringstream ls(line);
        std::string kind;
        ls >> kind;
        if (kind == "t") {
            double mean, var, ref, alpha;
            int n, k;
            ls >> mean >> var >> ref >> n >> alpha >> k;
            out << (hypothesis::students_t_test(mean, var, ref, n, alpha, k).first ? 1 : 0) << "\n";
        } else if (kind == "chi2") {
            std::string file;
            int cells, n, k;
            double min_exp, alpha;
            ls >> file >> cells >> n >> min_exp >> alpha >> k;
            std::vector<double> f(2 * (size_t)cells);
            std::ifstream fb(file, std::ios::binary);
            if (!fb.read(reinterpret_cast<char *>(f.data()), (std::streamsize)(f.size() * sizeof(double)))) return 3;
            out << (hypothesis::chi2_test(cells, f.data(), f.data() + cells, n, min_exp, alpha, k).first ? 1 : 0)
                << "\n";
        } else if (!kind.empty()) {
            return 2;
        }
    }
    return 0;
}
