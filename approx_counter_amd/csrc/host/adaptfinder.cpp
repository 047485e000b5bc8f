// adaptfinder.cpp -- the drop-in command line (binary `adaptFinder`).
//
// Same flags, config file, precedence, defaults, messages and output files as
// qbonenfant/approx_counter's main (approx_counter.cpp:604-958), so that
// Porechop_ABI can run it unchanged.  The approximate count (errorCount,
// approx_counter.cpp:531-601) goes through the C ABI of
// include/approx_counter_amd.h to the HIP kernel; there is no CPU fallback.
//
// Extensions (not in the reference, documented in DESIGN.md):
//   -g, --gpus N    shard the sampled windows over N GPUs of this node (default 1)
//   --seed N        seed the read sampling (the reference always uses std::random_device)
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <future>
#include <iostream>
#include <map>
#include <random>
#include <stdexcept>
#include <string>
#include <vector>

#include "approx_counter_amd.h"
#include "host_stages.h"

using namespace achost;

namespace {

const auto boot_time = std::chrono::steady_clock::now();

// print (approx_counter.cpp:85-94)
template <typename T>
void print(const T& text, int tab = 0) {
    const double ms = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - boot_time).count();
    std::cout << "[" << ms << " ms]\t";
    for (int i = 0; i < tab; ++i) std::cout << "\t";
    std::cout << text << std::endl;
}

// ---------------------------------------------------------------------------
// Argument parsing with the SeqAn ArgumentParser spellings (get_args, 604-669)
// ---------------------------------------------------------------------------
enum class Kind { Int, Double, String, Flag };
struct Opt {
    const char* s;
    const char* l;
    Kind kind;
    const char* help;
};
const Opt OPTS[] = {
    {"lc", "low_complexity", Kind::Double, "low complexity filter threshold (for k=16), default 1.5"},
    {"sn", "sample_n", Kind::Int, "sample n sequences from dataset, default 10k sequences"},
    {"sl", "sample_length", Kind::Int, "size of the sampled portion, default 100 bases"},
    {"nt", "nb_thread", Kind::Int, "Number of thread to work with, default is 4"},
    {"k", "kmer_size", Kind::Int, "Size of the kmers, default is 16"},
    {"lim", "limit", Kind::Int, "limit the number of kmer used after initial counting, default is 500"},
    {"mr", "multi_run", Kind::Int, "Number of time the count must be performed. Each count is exported separately."},
    {"v", "verbosity", Kind::Int, "Level of details printed out"},
    {"e", "exact_file", Kind::String, "path to export the exact k-mer count, if needed. Default: no export"},
    {"conf", "config", Kind::String, "path to the config file"},
    {"fk", "forbidden_kmer", Kind::String,
     "take a file containing 'forbidden' kmers, excluding them from the search pool. One kmer per line."},
    {"sk", "solid_km", Kind::Int,
     "Use solid kmer instead of most frequents. This option will override sample number (-sn / --sample_n)."},
    {"se", "skip_end", Kind::Flag,
     "Skip end adapter ressearch (only search start). /!\\ If this option is set, and adaptFinder is run trough "
     "PorechopABI, the --guess_only / -go MUST be set."},
    {"o", "out_file", Kind::String, "path to the output file, default is ./out.txt"},
    {"g", "gpus", Kind::Int, "[MI355X build] number of GPUs of this node to shard the count over, default 1"},
    {"", "seed", Kind::Int, "[MI355X build] seed of the read sampling, default: std::random_device"},
    {"", "host-exact", Kind::Flag,
     "[MI355X build] the reference's host stages: whole reads in memory, exact k-mer count on the CPU"},
    {"", "dump-sample", Kind::String,
     "[MI355X build] write each sampled window image to <path>_<run>.<end> and stop before counting"},
};

struct Args {
    std::map<std::string, std::string> val;  // by long name
    std::string input;
};

void usage(std::ostream& os) {
    os << "adaptFinder\n===========\n\nSYNOPSIS\n    adaptFinder [OPTIONS] \"input filename\"\n\n"
          "REQUIRED ARGUMENTS\n    input filename STRING\n\nOPTIONS\n    -h, --help\n          Display the help message.\n";
    for (const Opt& o : OPTS) {
        os << "    ";
        if (*o.s) os << "-" << o.s << ", ";
        os << "--" << o.l;
        switch (o.kind) {
            case Kind::Int: os << " INTEGER"; break;
            case Kind::Double: os << " DOUBLE"; break;
            case Kind::String: os << " STRING"; break;
            case Kind::Flag: break;
        }
        os << "\n          " << o.help << "\n";
    }
}

bool valid_value(Kind kind, const std::string& v) {
    if (v.empty()) return false;
    char* end = nullptr;
    if (kind == Kind::Int) {
        std::strtoll(v.c_str(), &end, 10);
        return *end == '\0';
    }
    if (kind == Kind::Double) {
        std::strtod(v.c_str(), &end);
        return *end == '\0';
    }
    return true;
}

// Returns 0 = OK, 1 = parse error, 2 = help printed.
int parse_args(int argc, char const** argv, Args& a) {
    std::vector<std::string> positional;
    for (int i = 1; i < argc; ++i) {
        std::string t = argv[i];
        if (t == "-h" || t == "--help") {
            usage(std::cout);
            return 2;
        }
        if (t.size() > 1 && t[0] == '-' && !(t.size() > 1 && (std::isdigit((unsigned char)t[1]) || t[1] == '.'))) {
            std::string name = t.substr(t[1] == '-' ? 2 : 1), value;
            bool has_inline = false;
            const size_t eq = name.find('=');
            if (eq != std::string::npos) {
                value = name.substr(eq + 1);
                name = name.substr(0, eq);
                has_inline = true;
            }
            const Opt* opt = nullptr;
            for (const Opt& o : OPTS)
                if ((t[1] == '-' && name == o.l) || (t[1] != '-' && *o.s && name == o.s)) opt = &o;
            if (!opt) {
                std::cerr << "adaptFinder: illegal option -- " << name << "\n";
                return 1;
            }
            if (opt->kind == Kind::Flag) {
                a.val[opt->l] = "1";
                continue;
            }
            if (!has_inline) {
                if (i + 1 >= argc) {
                    std::cerr << "adaptFinder: option requires an argument -- " << name << "\n";
                    return 1;
                }
                value = argv[++i];
            }
            if (!valid_value(opt->kind, value)) {
                std::cerr << "adaptFinder: the given value '" << value << "' cannot be casted to "
                          << (opt->kind == Kind::Int ? "integer" : "double") << "\n";
                return 1;
            }
            a.val[opt->l] = value;
        } else {
            positional.push_back(t);
        }
    }
    if (positional.size() != 1) {
        std::cerr << "adaptFinder: " << (positional.empty() ? "Not enough" : "Too many") << " arguments given.\n";
        return 1;
    }
    a.input = positional[0];
    return 0;
}

template <typename T>
void get_option(const Args& a, const char* long_name, T& out);
template <>
void get_option(const Args& a, const char* n, uint64_t& out) {
    auto it = a.val.find(n);
    if (it != a.val.end()) out = (uint64_t)std::strtoll(it->second.c_str(), nullptr, 10);
}
template <>
void get_option(const Args& a, const char* n, float& out) {
    auto it = a.val.find(n);
    if (it != a.val.end()) out = (float)std::strtod(it->second.c_str(), nullptr);
}
template <>
void get_option(const Args& a, const char* n, std::string& out) {
    auto it = a.val.find(n);
    if (it != a.val.end()) out = it->second;
}

// ---------------------------------------------------------------------------
// errorCount (approx_counter.cpp:531-601) through the C ABI, windows sharded
// over n_gpus devices (contiguous ranges balanced by bases), counts summed.
// ---------------------------------------------------------------------------
ac_windows view(const PackedImage& p) {
    return ac_windows{p.codes.data(), p.nmask.data(), p.start.data(), p.length.data(), (uint32_t)p.size(), p.n_bases};
}

// The device context: -g N opens N shards (device g mod the visible devices,
// ac_create_multi); the exact count and the one-GPU approximate count use the
// first device, the sharded count goes through ac_error_count_images.
struct Devices {
    ac_ctx* ctx = nullptr;
    uint64_t shards = 1;
    ~Devices() { ac_destroy(ctx); }
};

// --dump-sample: u64 n_windows, u64 n_bases, start[n] u64, length[n] u32,
// codes[n_bases/16] u32, nmask[n_bases/32] u32 (little endian).
bool write_image(const PackedImage& p, const std::string& path) {
    std::FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) return false;
    const uint64_t hdr[2] = {p.size(), p.n_bases};
    bool ok = std::fwrite(hdr, sizeof hdr, 1, f) == 1;
    ok = ok && std::fwrite(p.start.data(), sizeof(uint64_t), p.size(), f) == p.size();
    ok = ok && std::fwrite(p.length.data(), sizeof(uint32_t), p.size(), f) == p.size();
    ok = ok && std::fwrite(p.codes.data(), sizeof(uint32_t), p.codes.size(), f) == p.codes.size();
    ok = ok && std::fwrite(p.nmask.data(), sizeof(uint32_t), p.nmask.size(), f) == p.nmask.size();
    return std::fclose(f) == 0 && ok;
}

void open_devices(Devices& dev, uint64_t n_gpus) {
    if (dev.ctx) return;
    if (n_gpus < 1) n_gpus = 1;
    const int n_dev = ac_device_count();
    if (n_dev < 1) throw std::runtime_error("no HIP device available (the approximate count runs on the GPU only)");
    if ((int)n_gpus > n_dev)
        std::cerr << "/!\\ WARNING: " << n_gpus << " shards requested on " << n_dev << " visible GPU(s)\n";
    if (ac_create_multi(&dev.ctx, (int)n_gpus) != AC_OK) throw std::runtime_error(ac_last_error(nullptr));
    dev.shards = n_gpus;
}

// count_kmers + get_most_frequent / get_solid_kmers (approx_counter.cpp:874-899)
// on the GPU over a sample already uploaded to ctx (ac_exact_count_device).
pair_vector exact_count_gpu(ac_ctx* ctx, const ac_windows& dsample, uint32_t k, float lc, const kmer_set& forbidden,
                            uint64_t limit, uint64_t solid, uint64_t* n_distinct, uint64_t* had_n) {
    std::vector<uint64_t> fb(forbidden.begin(), forbidden.end());
    // Start small: a huge -lim (used to mean "keep all") must not allocate
    // `limit` entries up front; the call reports the size it needs.
    uint64_t cap = std::max<uint64_t>(1, solid ? 4096 : std::min<uint64_t>(limit, 4096));
    for (;;) {
        std::vector<uint64_t> km(cap), ct(cap);
        uint64_t n_out = 0;
        const ac_status st = ac_exact_count_device(ctx, k, &dsample, lc, fb.data(), (uint32_t)fb.size(), limit, solid,
                                                   km.data(), ct.data(), cap, &n_out, n_distinct, had_n);
        if (st == AC_ERR_INVALID && n_out > cap) {  // more kept k-mers than room
            cap = n_out;
            continue;
        }
        if (st != AC_OK) throw std::runtime_error(std::string("exact count failed: ") + ac_last_error(ctx));
        pair_vector out(n_out);
        for (uint64_t i = 0; i < n_out; ++i) out[i] = {km[i], ct[i]};
        return out;
    }
}

}  // namespace

int main(int argc, char const** argv) {
    Args args;
    const int pr = parse_args(argc, argv, args);
    if (pr != 0) return pr == 1;

    // Defaults (approx_counter.cpp:700-715)
    std::string output = "out.txt", exact_out, config_file, forbid_kmer;
    uint64_t solid_km = 0, nb_thread = 4, k = 16, sl = 100, sn = 40000, limit = 500, v = 1, nb_of_runs = 1;
    float param_lc = 1.0f, lc = 1.0f;
    bool skip_end = false;
    uint64_t n_gpus = 1;
    std::string seed_str;

    // Config file (721-737): CLI > config > defaults
    get_option(args, "config", config_file);
    if (!config_file.empty()) {
        bool opened = false;
        arg_map p = parse_config(config_file, &opened);
        if (!opened) std::cerr << "/!\\ WARNING: Could not open config file\n";
        param_lc = p.count("lc") ? std::stof(p["lc"]) : lc;
        k = p.count("k") ? std::stoi(p["k"]) : k;
        v = p.count("v") ? std::stoi(p["v"]) : v;
        sn = p.count("sn") ? std::stoi(p["sn"]) : sn;
        sl = p.count("sl") ? std::stoi(p["sl"]) : sl;
        limit = p.count("lim") ? std::stoi(p["lim"]) : limit;
        nb_thread = p.count("nt") ? std::stoi(p["nt"]) : nb_thread;
        solid_km = p.count("sk") ? std::stoi(p["sk"]) : solid_km;
        skip_end = p.count("se") > 0;
        forbid_kmer = p.count("fk") ? p["fk"] : forbid_kmer;
        exact_out = p.count("e") ? p["e"] : exact_out;
        nb_of_runs = p.count("mr") ? std::stoi(p["mr"]) : nb_of_runs;
    }
    get_option(args, "limit", limit);
    get_option(args, "low_complexity", param_lc);
    get_option(args, "kmer_size", k);
    get_option(args, "verbosity", v);
    get_option(args, "sample_length", sl);
    get_option(args, "sample_n", sn);
    get_option(args, "nb_thread", nb_thread);
    get_option(args, "out_file", output);
    get_option(args, "exact_file", exact_out);
    get_option(args, "forbidden_kmer", forbid_kmer);
    get_option(args, "solid_km", solid_km);
    get_option(args, "multi_run", nb_of_runs);
    get_option(args, "gpus", n_gpus);
    get_option(args, "seed", seed_str);
    skip_end = skip_end || args.val.count("skip_end");
    const bool host_exact = args.val.count("host-exact") > 0;
    std::string dump_sample;
    get_option(args, "dump-sample", dump_sample);
    const std::string input_file = args.input;

    kmer_set forbidden;
    if (!forbid_kmer.empty()) {
        print("Parsing the fobidden kmer list");
        if (!parse_kmer_list(forbid_kmer, forbidden)) {
            std::cerr << "/!\\ ERROR: COULD NOT OPEN EXCLUDED KMER FILE, must quit\n";
            std::exit(1);
        }
    }
    const int mr_v = (nb_of_runs > 1 && v < 2) ? 0 : (int)v;
    const std::string warning = "/!\\ WARNING: ", error_pref = "/!\\ ERROR: ";
    if (k < 2 || k > 32) throw std::invalid_argument(error_pref + "kmer size must be between 2 and 32 (included)");
    if (k > sl) throw std::invalid_argument(error_pref + "kmer size must be smaller than the sampling length (k <= sl)");
    lc = adjust_threshold(param_lc, 16, (uint32_t)k);

    if (v > 0) {
        std::cout << "Kmer size:             " << k << std::endl;
        std::cout << "Sampled sequences:     " << sn << std::endl;
        std::cout << "Sampling length        " << sl << std::endl;
        std::cout << "LC filter threshold:   " << param_lc << std::endl;
        std::cout << "Adjusted LC threshold: " << lc << std::endl;
        std::cout << "Nb thread:             " << nb_thread << std::endl;
        if (solid_km != 0) std::cout << "Solid kmers:           " << solid_km << std::endl;
        else std::cout << "Number of kept kmer:   " << limit << std::endl;
        std::cout << "Number of runs:        " << nb_of_runs << std::endl;
        std::cout << "Verbosity level:       " << v << std::endl;
    }
    int tab_level = 0;
    if (v > 0 && nb_of_runs > 1) std::cout << "\nA total of " << nb_of_runs << " runs will be performed." << std::endl;

    // Reads: by default only their sampling windows are kept, packed while the
    // file is parsed (read_windows); --host-exact keeps whole reads as the
    // reference does.  Both throw (uncaught, like SeqAn's IOError) on an
    // unreadable file.
    std::vector<std::string> ids;
    SeqSet seqs;
    WindowStore store;
    // The GPU contexts (the reference builds its index inside errorCount; the
    // device set is opened once).  Opening them (HIP runtime + device
    // initialisation, ~75 ms) runs on a helper thread while the input is parsed;
    // the first GPU stage waits for it and reports its failure, if any.
    Devices dev;
    std::future<void> dev_ready;
    if (dump_sample.empty()) dev_ready = std::async(std::launch::async, [&dev, n_gpus] { open_devices(dev, n_gpus); });
    auto devices = [&]() {
        if (dev_ready.valid()) dev_ready.get();  // rethrows the helper's exception
        open_devices(dev, n_gpus);
    };
    if (v > 0) print("Parsing FASTA file", tab_level);
    if (host_exact) read_records(input_file, ids, seqs);
    else read_windows(input_file, sl, store);
    const uint64_t n_reads = host_exact ? seqs.size() : store.size();
    if (v > 0) print("Number of sequences found: " + std::to_string(n_reads) + ".", tab_level);

    std::mt19937 rng(seed_str.empty() ? std::random_device{}() : (uint32_t)std::strtoull(seed_str.c_str(), nullptr, 10));

    // One run samples both read ends, counts each end's k-mers exactly, then counts both
    // ends approximately in ONE fused launch (errorCount, approx_counter.cpp:922, for the
    // two iterations of the loop at 858-953, whose inputs are independent), and ranks and
    // exports each end.  Output files and their contents are the reference's; only the
    // order of the progress messages differs.
    struct End {
        std::string which;
        PackedImage img;
        ac_windows dsample{};
        pair_vector first_n;
    };
    for (uint64_t run = 0; run < nb_of_runs; ++run) {
        const std::string run_suffix = "_" + std::to_string(run);
        if (nb_of_runs > 1 && v > 0) std::cout << "Starting run number " << run + 1 << std::endl;
        if (sn > n_reads) {
            std::cerr << warning << "Sequence set too small for the requested sample size\n";
            std::cerr << warning << "The whole set will be used.\n";
            sn = n_reads;
        }
        bool bottom = false;
        tab_level += 1;
        std::vector<End> pending;
        // the approximate count of the pending ends, then their ranking and export
        auto flush = [&]() -> bool {
            if (pending.empty()) return true;
            std::vector<std::vector<uint64_t>> km(pending.size()), ct(pending.size());
            std::vector<ac_sample_job> jobs(pending.size());
            for (size_t e = 0; e < pending.size(); ++e) {
                if (mr_v > 0) print("Approximate k-mer count (" + pending[e].which + ")", tab_level);
                for (const auto& x : pending[e].first_n) km[e].push_back(x.first);
                ct[e].assign(km[e].size(), 0);
                jobs[e] = ac_sample_job{km[e].data(), (uint32_t)km[e].size(), ac_windows{}, ct[e].data()};
            }
            try {
                devices();
                const bool on_device = !host_exact && dev.shards == 1;  // the samples uploaded for the exact count
                for (size_t e = 0; e < pending.size(); ++e)
                    jobs[e].sample = on_device ? pending[e].dsample : view(pending[e].img);
                const ac_status st =
                    on_device ? ac_error_count_samples(dev.ctx, (uint32_t)k, jobs.data(), (uint32_t)jobs.size())
                              : ac_error_count_images(dev.ctx, (uint32_t)k, jobs.data(), (uint32_t)jobs.size());
                if (st != AC_OK) throw std::runtime_error(ac_last_error(dev.ctx));
            } catch (const std::exception& e) {
                std::cerr << error_pref << "approximate count failed: " << e.what() << std::endl;
                return false;
            }
            for (size_t e = 0; e < pending.size(); ++e) {
                pair_vector error_counter(km[e].size());
                for (size_t i = 0; i < km[e].size(); ++i) error_counter[i] = {km[e][i], ct[e][i]};
                pair_vector sorted_error_count = get_most_frequent(std::move(error_counter), limit, (uint32_t)k);
                if (mr_v > 0) print("Exporting approximate count", tab_level);
                const std::string path = output + run_suffix + "." + pending[e].which;
                if (!export_counter(sorted_error_count, (uint32_t)k, path)) {
                    std::cerr << error_pref + "Failed to export approximate k-mer count" << std::endl;
                    std::cerr << "Path: " << path << std::endl;
                    return false;
                }
                if (mr_v > 0) print("Done", tab_level);
            }
            pending.clear();
            return true;
        };
        for (const std::string which_end : {"start", "end"}) {
            if (v > 0) print("Working on sequence " + which_end + ".", tab_level - 1);
            if (mr_v > 0) print("Sampling", tab_level);
            if (mr_v > 0) print(bottom ? "Sampling the ends of reads" : "Sampling the start of reads", 1);
            End cur;
            cur.which = which_end;
            SeqSet sample;
            if (host_exact) {
                sample = sample_sequences(seqs, sn, sl, bottom, rng);
                cur.img = pack_sample(sample, 0, sample.size());
            } else {
                cur.img = sample_windows(store, sn, bottom, rng);
            }
            if (mr_v > 0) print("Sampled " + std::to_string(cur.img.size()) + " sequences", 1);
            if (!dump_sample.empty()) {
                if (!write_image(cur.img, dump_sample + run_suffix + "." + which_end)) {
                    std::cerr << error_pref << "could not write " << dump_sample + run_suffix + "." + which_end << "\n";
                    return 1;
                }
                if (!skip_end) bottom = true;
                else if (mr_v > 0) break;  // the -se quirk below
                continue;
            }
            if (mr_v > 0) print("Exact k-mer count", tab_level);
            uint64_t had_n = 0, n_found = 0;
            if (host_exact) {  // the reference's host stages (approx_counter.cpp:874-899)
                pair_vector count = count_kmers(sample, (uint32_t)k, lc, forbidden, &had_n);
                n_found = count.size();
                cur.first_n = solid_km != 0 ? get_solid_kmers(std::move(count), solid_km, (uint32_t)k)
                                            : get_most_frequent(std::move(count), limit, (uint32_t)k);
            } else {  // the same on GPU 0; the upload (one slot per end) also serves the approximate count
                try {
                    devices();
                    const ac_windows hw = view(cur.img);
                    if (ac_sample_upload_slot(dev.ctx, (int)pending.size(), &hw, &cur.dsample) != AC_OK)
                        throw std::runtime_error(ac_last_error(dev.ctx));
                    cur.first_n = exact_count_gpu(dev.ctx, cur.dsample, (uint32_t)k, lc, forbidden, limit, solid_km,
                                                  &n_found, &had_n);
                } catch (const std::exception& e) {
                    std::cerr << error_pref << "exact count failed: " << e.what() << std::endl;
                    // the reference exported the earlier end's approximate count before reaching this end
                    // (ADVICE r3): its own upload slot is intact, so count and write it first
                    flush();
                    return 1;
                }
            }
            if (had_n > 0) {
                std::cerr << "/!\\ WARNING: This dataset contained sequences with 'N' symbols. ";
                std::cerr << "/!\\ WARNING: Current implementation ignores k-mers containing 'N'.";
                std::cerr << "/!\\ WARNING: A total of " << had_n << " k-mers were ignored." << std::endl;
            }
            if (mr_v > 0) print("Number of kmer found: " + std::to_string(n_found), tab_level);
            if (mr_v > 0) print(solid_km != 0 ? "Keeping solid k-mer" : "Keeping most frequent k-mer", tab_level);
            if (mr_v > 0) print("Number of kmer kept:  " + std::to_string(cur.first_n.size()), tab_level);
            if (!exact_out.empty()) {
                if (mr_v > 0) print("Exporting exact kmer count", tab_level);
                if (!export_counter(cur.first_n, (uint32_t)k, exact_out + run_suffix + "." + which_end)) {
                    std::cerr << error_pref + "Failed to export exact k-mer count" << std::endl;
                    std::cerr << "Path: " << exact_out + run_suffix + "." + which_end << std::endl;
                    flush();  // the reference wrote the earlier end's approximate count before failing here
                    return 1;
                }
            }
            pending.push_back(std::move(cur));
            // approx_counter.cpp:943-951: the break only happens when verbose
            // (without it the second pass samples read STARTS again and writes
            // them to the .end file -- kept for drop-in fidelity).
            if (skip_end) {
                if (mr_v > 0) {
                    print("Skipping end adapter ressearch");
                    break;
                }
            } else {
                bottom = true;
            }
        }
        if (!flush()) return 1;
        tab_level--;
    }
    return 0;
}
