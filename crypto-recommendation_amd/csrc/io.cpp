// io.cpp — the reference's input formats, host side.
//
//   VectorReader<T>::read      lib/in_out/vector_reader.hpp:54-85
//   split / split_convert      lib/utils.cpp:11-19, lib/utils.hpp:85-94
//   file_to_args               lib/utils.cpp:53-69
//   ArgParser::getFlagValue    lib/in_out/arg_parser.cpp:21-33
//   get_config                 main.cpp:512-554
//
// The vector file is parsed in parallel: the byte range is cut at line
// boundaries into one slice per thread, each slice is parsed independently,
// and the rows are concatenated in file order. Values go through strtod (what
// std::stod calls), so every double is the reference's.
#include <algorithm>
#include <cerrno>
#include <cmath>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

#include "../../include/lshkm.h"
#include "common.h"

using namespace lshkm;

namespace {

struct Row {
    std::string id;
    std::vector<double> v;
};

// std::stod (libstdc++ __stoa): strtod, throwing invalid_argument when nothing
// parses and out_of_range whenever strtod sets ERANGE (overflow, underflow).
int stod_like(const std::string& s, double* out) {
    const char* b = s.c_str();
    char* e = nullptr;
    errno = 0;
    const double v = strtod(b, &e);
    if (e == b || errno == ERANGE) return -1;
    *out = v;
    return 0;
}

// std::stoi: strtol, then out_of_range outside int.
int stoi_like(const std::string& s, long* out) {
    const char* b = s.c_str();
    char* e = nullptr;
    errno = 0;
    const long v = strtol(b, &e, 10);
    if (e == b || errno == ERANGE || v > 2147483647L || v < -2147483647L - 1) return -1;
    *out = v;
    return 0;
}

// One line of the vector file (vector_reader.hpp:73-80): strip every '\r',
// the ID is the text before the first delimiter, the values follow, split
// with getline semantics (no token after a trailing delimiter). A line
// without a delimiter keeps its whole text as both ID and values, as
// substr(npos + 1) = substr(0) does in the reference.
int parse_line(std::string line, char delim, Row* row, std::string* err) {
    line.erase(std::remove(line.begin(), line.end(), '\r'), line.end());
    const size_t p = line.find(delim);
    row->id = line.substr(0, p);
    const std::string rest = line.substr(p == std::string::npos ? 0 : p + 1);
    row->v.clear();
    size_t i = 0;
    while (i < rest.size()) {
        size_t j = rest.find(delim, i);
        if (j == std::string::npos) j = rest.size();
        double v;
        const std::string tok = rest.substr(i, j - i);
        if (stod_like(tok, &v)) {
            *err = "value \"" + tok + "\" of vector \"" + row->id + "\": std::stod would throw";
            return -1;
        }
        row->v.push_back(v);
        i = j + 1;
    }
    return 0;
}

int read_file(const char* path, std::string* data) {
    std::ifstream f(path, std::ios::binary);
    if (!f.is_open()) return -1;
    f.seekg(0, std::ios::end);
    const std::streamoff n = f.tellg();
    f.seekg(0, std::ios::beg);
    data->resize((size_t)std::max<std::streamoff>(n, 0));
    if (n > 0) f.read(&(*data)[0], n);
    return 0;
}

// file_to_args(filename, delimiter): every line split with getline semantics
// ("a  b" gives "a", "", "b"; an empty line gives nothing).
std::vector<std::string> file_args(const std::string& data, char delim) {
    std::vector<std::string> args;
    std::istringstream in(data);
    std::string line;
    while (std::getline(in, line)) {
        std::istringstream ls(line);
        std::string tok;
        while (std::getline(ls, tok, delim)) args.push_back(tok);
    }
    return args;
}

// ArgParser::getFlagValue: the token after the first occurrence of the flag.
// (The reference constructs std::string(NULL) — undefined — when the flag is
// the last token; here that is "not found".)
const std::string* flag_value(const std::vector<std::string>& args, const std::string& flag) {
    auto it = std::find(args.begin(), args.end(), flag);
    if (it == args.end() || it + 1 == args.end()) return nullptr;
    return &*(it + 1);
}

void copy_str(const std::string& s, char* dst, size_t cap) {
    const size_t n = std::min(s.size(), cap - 1);
    std::memcpy(dst, s.data(), n);
    dst[n] = 0;
}

}  // namespace

struct lshkm_vectors_s {
    std::vector<std::string> meta;
    std::vector<Row> rows;
};

extern "C" {

int lshkm_vectors_read(const char* path, char delimiter, int strt_line, int threads, lshkm_vectors* out) {
    LSHKM_CHECK(path && out && strt_line >= 1, LSHKM_ERR_ARG, "bad arguments");
    std::string data;
    LSHKM_CHECK(read_file(path, &data) == 0, LSHKM_ERR_ARG, std::string("cannot open ") + path);
    lshkm_vectors v = new lshkm_vectors_s();
    // metadata lines 1 .. strt_line-1 (vector_reader.hpp:66-70)
    size_t pos = 0;
    for (int ln = 1; ln < strt_line && pos < data.size(); ln++) {
        size_t e = data.find('\n', pos);
        if (e == std::string::npos) e = data.size();
        v->meta.push_back(data.substr(pos, e - pos));
        pos = std::min(data.size(), e + 1);
    }
    int nt = threads > 0 ? threads : (int)std::max(1u, std::thread::hardware_concurrency());
    nt = std::min(nt, 64);
    const size_t body = data.size() - pos;
    if (body < ((size_t)1 << 20)) nt = 1;
    std::vector<size_t> cut(nt + 1, data.size());
    cut[0] = pos;
    for (int t = 1; t < nt; t++) {
        const size_t c = std::max(pos + body / nt * t, cut[t - 1]);
        const size_t e = c >= data.size() ? std::string::npos : data.find('\n', c);
        cut[t] = e == std::string::npos ? data.size() : e + 1;
    }
    std::vector<std::vector<Row>> part(nt);
    std::vector<std::string> errs(nt);
    auto work = [&](int t) {
        size_t p = cut[t];
        while (p < cut[t + 1]) {    // getline yields no line after a final '\n'
            size_t e = data.find('\n', p);
            if (e == std::string::npos || e > cut[t + 1]) e = cut[t + 1];
            Row r;
            if (parse_line(data.substr(p, e - p), delimiter, &r, &errs[t])) return;
            part[t].push_back(std::move(r));
            p = e + 1;
        }
    };
    std::vector<std::thread> pool;
    for (int t = 1; t < nt; t++) pool.emplace_back(work, t);
    work(0);
    for (auto& th : pool) th.join();
    for (int t = 0; t < nt; t++)
        if (!errs[t].empty()) { delete v; set_error(errs[t]); return LSHKM_ERR_ARG; }
    size_t total = 0;
    for (auto& p : part) total += p.size();
    v->rows.reserve(total);
    for (auto& p : part)
        for (auto& r : p) v->rows.push_back(std::move(r));
    *out = v;
    return 0;
}

int lshkm_vectors_info(lshkm_vectors v, int64_t* n, int* d, int64_t* id_bytes, int* ragged, int* fp32_exact,
                       int* n_meta) {
    LSHKM_CHECK(v, LSHKM_ERR_ARG, "vectors is NULL");
    const int64_t N = (int64_t)v->rows.size();
    const int D = N ? (int)v->rows[0].v.size() : 0;
    int64_t ib = 0;
    int rg = 0, ex = 1;
    for (const Row& r : v->rows) {
        ib += (int64_t)r.id.size();
        rg |= (int)r.v.size() != D;
        for (double x : r.v) ex &= (double)(float)x == x || x != x;
    }
    if (n) *n = N;
    if (d) *d = D;
    if (id_bytes) *id_bytes = ib;
    if (ragged) *ragged = rg;
    if (fp32_exact) *fp32_exact = ex;
    if (n_meta) *n_meta = (int)v->meta.size();
    return 0;
}

int lshkm_vectors_values(lshkm_vectors v, double* X64_host, float* X32_host) {
    LSHKM_CHECK(v, LSHKM_ERR_ARG, "vectors is NULL");
    const size_t D = v->rows.empty() ? 0 : v->rows[0].v.size();
    for (const Row& r : v->rows) LSHKM_CHECK(r.v.size() == D, LSHKM_ERR_STATE, "ragged rows: no N x d layout");
    for (size_t i = 0; i < v->rows.size(); i++)
        for (size_t j = 0; j < D; j++) {
            const double x = v->rows[i].v[j];
            if (X64_host) X64_host[i * D + j] = x;
            if (X32_host) X32_host[i * D + j] = (float)x;
        }
    return 0;
}

int lshkm_vectors_ids(lshkm_vectors v, char* bytes_host, int64_t* offsets_host) {
    LSHKM_CHECK(v && offsets_host && (bytes_host || v->rows.empty()), LSHKM_ERR_ARG, "bad arguments");
    int64_t o = 0;
    offsets_host[0] = 0;
    for (size_t i = 0; i < v->rows.size(); i++) {
        std::memcpy(bytes_host + o, v->rows[i].id.data(), v->rows[i].id.size());
        o += (int64_t)v->rows[i].id.size();
        offsets_host[i + 1] = o;
    }
    return 0;
}

int lshkm_vectors_meta(lshkm_vectors v, int index, char* buf, int64_t cap, int64_t* len) {
    LSHKM_CHECK(v && index >= 0, LSHKM_ERR_ARG, "bad arguments");
    // getMetaLine: "" past the saved lines (vector_reader.hpp:91-96)
    const std::string s = index < (int)v->meta.size() ? v->meta[index] : std::string();
    if (len) *len = (int64_t)s.size();
    if (buf && cap > 0) copy_str(s, buf, (size_t)cap);
    return 0;
}

int lshkm_vectors_free(lshkm_vectors v) {
    delete v;
    return 0;
}

int lshkm_config_value(const char* path, const char* key, char* buf, int64_t cap, int* found) {
    LSHKM_CHECK(path && key && found, LSHKM_ERR_ARG, "bad arguments");
    std::string data;
    *found = 0;
    if (read_file(path, &data)) return 0;   // file_to_args: no file -> no arguments
    const std::vector<std::string> args = file_args(data, ' ');
    const std::string* v = flag_value(args, key);
    if (!v) return 0;
    *found = 1;
    if (buf && cap > 0) copy_str(*v, buf, (size_t)cap);
    return 0;
}

int lshkm_config_load(const char* path, lshkm_config* c) {
    LSHKM_CHECK(path && c, LSHKM_ERR_ARG, "bad arguments");
    std::memset(c, 0, sizeof(*c));
    // main.cpp:50-63 defaults
    c->proj_2_csv_delimiter = ' ';
    c->proj_2_cluster_num = 100;
    c->k = 4;
    c->L = 5;
    c->lsh_bucket_div = 4;
    c->euclidean_h_w = 0.01;
    c->max_algo_iterations = 30;
    c->min_dist_kmeans = 0.05;
    c->csv_delimiter = ' ';
    std::string data;
    if (read_file(path, &data)) data.clear();
    const std::vector<std::string> args = file_args(data, ' ');
    auto num_i = [&](const char* k, int* dst) -> int {
        const std::string* v = flag_value(args, k);
        if (!v) return 0;
        long x;
        LSHKM_CHECK(stoi_like(*v, &x) == 0, LSHKM_ERR_ARG, std::string("config ") + k + ": stoi(\"" + *v + "\") throws");
        *dst = (int)x;
        return 0;
    };
    auto num_d = [&](const char* k, double* dst) -> int {
        const std::string* v = flag_value(args, k);
        if (!v) return 0;
        LSHKM_CHECK(stod_like(*v, dst) == 0, LSHKM_ERR_ARG, std::string("config ") + k + ": stod(\"" + *v + "\") throws");
        return 0;
    };
    int rc;
    // number_of_clusters is required: main.cpp:518-523 asks on stdin otherwise
    c->has_cluster_num = flag_value(args, "number_of_clusters") != nullptr;
    if ((rc = num_i("number_of_clusters", &c->cluster_num))) return rc;
    if (const std::string* v = flag_value(args, "proj_2_input")) copy_str(*v, c->proj_2_input, sizeof(c->proj_2_input));
    if (const std::string* v = flag_value(args, "proj_2_csv_delimiter")) c->proj_2_csv_delimiter = v->empty() ? 0 : (*v)[0];
    if ((rc = num_i("proj_2_number_of_clusters", &c->proj_2_cluster_num)) || (rc = num_i("number_of_hash_functions", &c->k)) ||
        (rc = num_i("number_of_hash_tables", &c->L)) || (rc = num_i("lsh_bucket_div", &c->lsh_bucket_div)) ||
        (rc = num_d("euclidean_h_w", &c->euclidean_h_w)) ||
        (rc = num_i("max_algo_iterations", &c->max_algo_iterations)) || (rc = num_d("min_dist_kmeans", &c->min_dist_kmeans)))
        return rc;
    if (flag_value(args, "csv_delimiter")) {
        int code = 0;
        if ((rc = num_i("csv_delimiter", &code))) return rc;
        c->csv_delimiter = (char)code;            // an ASCII code (main.cpp:544-547)
    }
    if (const std::string* v = flag_value(args, "lexicon_file")) copy_str(*v, c->lexicon_file, sizeof(c->lexicon_file));
    if (const std::string* v = flag_value(args, "query_file")) copy_str(*v, c->query_file, sizeof(c->query_file));
    return 0;
}

}  // extern "C"
