// host_asan.cpp — the host-side parsers of liblshkm (csrc/io.cpp: the CSV
// vector reader, cluster.conf / file_to_args, ArgParser) built with
// -fsanitize=address,undefined on the host side only, and run over the
// committed format fixtures plus generated malformed inputs (truncated lines,
// empty tokens, huge and ragged rows, NUL bytes, missing files). Driven by
// tests/test_host_asan.py; any sanitizer report fails the run.
#include <cstdio>
#include <cstdlib>
#include <random>
#include <string>
#include <vector>

#include "../crypto-recommendation_amd/csrc/io.cpp"

namespace lshkm {
static std::string g_err;
void set_error(const std::string& msg) { g_err = msg; }
}  // namespace lshkm

static int read_all(const char* path, char delim, int strt, int threads) {
    lshkm_vectors v = nullptr;
    const int rc = lshkm_vectors_read(path, delim, strt, threads, &v);
    if (rc) return rc;
    int64_t n = 0, idb = 0;
    int d = 0, ragged = 0, fp32 = 0, nmeta = 0;
    lshkm_vectors_info(v, &n, &d, &idb, &ragged, &fp32, &nmeta);
    std::vector<double> x64((size_t)std::max<int64_t>(n * d, 1));
    std::vector<float> x32((size_t)std::max<int64_t>(n * d, 1));
    std::vector<char> ids((size_t)std::max<int64_t>(idb, 1));
    std::vector<int64_t> off((size_t)n + 1);
    if (!ragged) lshkm_vectors_values(v, x64.data(), x32.data());
    lshkm_vectors_ids(v, ids.data(), off.data());
    char buf[256];
    int64_t len = 0;
    for (int i = 0; i < nmeta; i++) lshkm_vectors_meta(v, i, buf, sizeof buf, &len);
    lshkm_vectors_free(v);
    return 0;
}

static void write_file(const char* path, const std::string& s) {
    FILE* f = fopen(path, "wb");
    fwrite(s.data(), 1, s.size(), f);
    fclose(f);
}

int main(int argc, char** argv) {
    // argv: tmpdir, then fixture files (csv or conf)
    if (argc < 2) return 2;
    const std::string tmp = argv[1];
    for (int i = 2; i < argc; i++) {
        const std::string p = argv[i];
        if (p.size() > 5 && p.substr(p.size() - 5) == ".conf") {
            lshkm_config c;
            lshkm_config_load(p.c_str(), &c);
            char buf[64];
            int found = 0;
            lshkm_config_value(p.c_str(), "number_of_clusters", buf, sizeof buf, &found);
            lshkm_config_value(p.c_str(), "no_such_key", buf, 1, &found);
        } else {
            for (int t : {1, 3, 8})
                for (char dl : {',', ' ', '\t'}) read_all(p.c_str(), dl, 1, t), read_all(p.c_str(), dl, 0, t);
        }
    }
    // malformed inputs
    std::mt19937 g(7);
    const char* alphabet = "0123456789.,-+eE \t\r\nabcinfINFnan#\x00";
    for (int it = 0; it < 300; it++) {
        std::string s;
        const int n = (int)(g() % 4000);
        for (int j = 0; j < n; j++) s.push_back(alphabet[g() % 34]);
        const std::string f = tmp + "/fuzz.csv";
        write_file(f.c_str(), s);
        read_all(f.c_str(), ',', (int)(g() % 3), 1 + (int)(g() % 8));
        const std::string c = tmp + "/fuzz.conf";
        write_file(c.c_str(), s);
        lshkm_config cc;
        lshkm_config_load(c.c_str(), &cc);
    }
    // structured edge cases
    const char* cases[] = {"", "\n", "id\n", "a,1,2\nb,3\n", "a,1,2,\nb,3,4,\n", "a,,,\n", "a,1e400,-1e-400\n",
                           "a,0x1p3,inf,nan\r\n", ",\n,\n", "a,1,2\n\n\nb,3,4"};
    for (const char* cs : cases) {
        const std::string f = tmp + "/case.csv";
        write_file(f.c_str(), cs);
        for (int t : {1, 2, 5}) read_all(f.c_str(), ',', 0, t), read_all(f.c_str(), ',', 1, t);
    }
    std::string wide = "w";
    for (int j = 0; j < 20000; j++) wide += ",1.5";
    wide += "\n";
    write_file((tmp + "/wide.csv").c_str(), wide + wide);
    read_all((tmp + "/wide.csv").c_str(), ',', 0, 4);
    read_all((tmp + "/missing_file.csv").c_str(), ',', 0, 1);
    puts("host_asan ok");
    return 0;
}
