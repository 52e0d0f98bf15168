// Shared command-line handling of bin/RS and bin/CPU-RS (reference CLI: src/main.c:32-167,
// README.md:29-50). Same short flags; uppercase aliases take their argument (the reference declares
// them argument-less and segfaults on atoi(NULL)); flags may come in any order;
// numeric arguments are validated (the reference divides by zero on -s 0).
#pragma once

#include <getopt.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

namespace gfrs_cli {

struct Args {
  enum Op { kNone, kEncode, kDecode, kMakeConf } op = kNone;
  int k = 0, n = 0;
  int grid = 0;     // -p: cap on gridDim.x (0 = uncapped)
  int streams = 1;  // -s
  std::string in_file, conf, out;
  std::string matrix = "vandermonde";
  std::string mul = "simd";
  int gpus = 0;  // 0 = all visible
  std::vector<int> devices;  // --devices 0,1,...: explicit shard -> device list (entries may repeat)
  int threads = 1;
  long long slice = 16ll << 20;
  bool cpu_meta = false;
  bool quiet = false;
  long long window = -1;  // --window: stream in column windows of this many bytes (0 = auto)
  bool resume = true;     // --no-resume: ignore a <target>.PROGRESS checkpoint
  bool sync = true;       // --no-sync: skip fdatasync before each checkpoint
  int field_w = 8;        // -w 8|16: symbol width (GF(2^8), or GF(2^16) for n up to 65535)
  // 1: the GEMM kernel reads / writes the pinned host rows over PCIe itself (no staging), 0: the
  // staged -s stream pipeline; -1 (default): zero-copy unless -s or --slice asked for streams
  int zero_copy = -1;
  bool streaming() const { return window >= 0; }
};

inline void usage(const char* prog, bool gpu) {
  std::printf("Usage:\n");
  std::printf("[-h]: show usage information\n");
  std::printf("Encode: [-k|-K nativeBlockNum] [-n|-N totalBlockNum] [-e|-E fileName]\n");
  std::printf("Decode: [-d|-D] [-k|-K nativeBlockNum] [-n|-N totalBlockNum] \n\t [-i|-I originalFileName] "
              "[-c|-C config] [-o|-O output]\n");
  std::printf("For encoding, the -k, -n, and -e options are all necessary.\n");
  std::printf("For decoding, the -d, -i, and -c options are all necessary.\n");
  std::printf("If the -o option is not set, the original file name will be chosen as the output file name by "
              "default.\n");
  if (gpu) {
    std::printf("Performance-tuning Options:\n");
    std::printf("[-p|-P]: set maximum gridDim.x (0 = one block per 4 KiB column group)\n");
    std::printf("[-s|-S]: set stream number\n");
  }
  std::printf("Extensions:\n");
  std::printf("  --matrix vandermonde|cauchy|sys_vandermonde  coding matrix (default: reference Vandermonde)\n");
  std::printf("  -w|-W 8|16              encode: symbol width, GF(2^8) (default) or GF(2^16) (n <= 65535;\n");
  std::printf("                          src/galoisfield.cu's w = 16 field); decode reads it from the METADATA\n");
  std::printf("  --cpu-meta              write the 2-line CPU-format METADATA\n");
  std::printf("  --make-conf             write conf-<n>-<k>-<file> keeping the last k chunks (unit-test.sh)\n");
  std::printf("  --window BYTES          bounded-memory streaming codec: column windows of BYTES per chunk\n");
  std::printf("                          (0 = auto), checkpointed to <target>.PROGRESS and resumable\n");
  std::printf("  --no-resume             with --window: start over even if a checkpoint matches\n");
  std::printf("  --no-sync               with --window: do not fdatasync before each checkpoint\n");
  std::printf("  -q                      quiet\n");
  if (gpu) {
    std::printf("  --gpus N                number of GPUs (default: all visible)\n");
    std::printf("  --devices I,J,...       explicit column-shard -> device list (a device may repeat)\n");
    std::printf("  --slice BYTES           column slice per stream step (default 16 MiB)\n");
    std::printf("  --zero-copy             (default unless -s or --slice is given) the GEMM kernel streams the\n");
    std::printf("                          pinned host rows itself over PCIe: no device slice buffers or copy engines\n");
    std::printf("  --staged                the -s stream pipeline: H2D copies into device slices, kernel, D2H\n");
  } else {
    std::printf("  --mul logexp|logexp0|logexp1|logexp2|logexp3|loop|full|double|perm|row|simd\n");
    std::printf("  --threads T             worker threads (default 1, the reference's single thread)\n");
  }
  (void)prog;
}

inline int to_int(const char* s, const char* what, int lo) {
  char* end = nullptr;
  const long v = std::strtol(s ? s : "", &end, 10);
  if (!s || *end || v < lo) {
    std::fprintf(stderr, "invalid %s: %s\n", what, s ? s : "(null)");
    std::exit(2);
  }
  return int(v);
}

inline long long to_ll(const char* s, const char* what, long long lo) {
  char* end = nullptr;
  const long long v = std::strtoll(s ? s : "", &end, 10);
  if (!s || *end || v < lo) {
    std::fprintf(stderr, "invalid %s: %s\n", what, s ? s : "(null)");
    std::exit(2);
  }
  return v;
}

inline Args parse(int argc, char** argv, bool gpu) {
  Args a;
  bool streams_given = false;
  static const option longopts[] = {{"matrix", required_argument, nullptr, 1},
                                    {"cpu-meta", no_argument, nullptr, 2},
                                    {"gpus", required_argument, nullptr, 3},
                                    {"slice", required_argument, nullptr, 4},
                                    {"mul", required_argument, nullptr, 5},
                                    {"threads", required_argument, nullptr, 6},
                                    {"make-conf", no_argument, nullptr, 7},
                                    {"window", required_argument, nullptr, 8},
                                    {"no-resume", no_argument, nullptr, 9},
                                    {"no-sync", no_argument, nullptr, 10},
                                    {"devices", required_argument, nullptr, 11},
                                    {"field-width", required_argument, nullptr, 'w'},
                                    {"zero-copy", no_argument, nullptr, 12},
                                    {"staged", no_argument, nullptr, 13},
                                    {"help", no_argument, nullptr, 'h'},
                                    {nullptr, 0, nullptr, 0}};
  int c;
  while ((c = getopt_long(argc, argv, "k:K:n:N:e:E:i:I:c:C:o:O:p:P:s:S:w:W:dDhq", longopts, nullptr)) != -1) {
    switch (c) {
      case 'k': case 'K': a.k = to_int(optarg, "nativeBlockNum", 1); break;
      case 'n': case 'N': a.n = to_int(optarg, "totalBlockNum", 1); break;
      case 'e': case 'E': a.op = a.op == Args::kMakeConf ? a.op : Args::kEncode; a.in_file = optarg; break;
      case 'd': case 'D': a.op = Args::kDecode; break;
      case 'i': case 'I': a.in_file = optarg; break;
      case 'c': case 'C': a.conf = optarg; break;
      case 'o': case 'O': a.out = optarg; break;
      case 'p': case 'P': a.grid = to_int(optarg, "grid size", 0); break;
      case 's': case 'S': a.streams = to_int(optarg, "stream number", 1); streams_given = true; break;
      case 'q': a.quiet = true; break;
      case 'w': case 'W':
        a.field_w = to_int(optarg, "field width", 8);
        if (a.field_w != 8 && a.field_w != 16) {
          std::fprintf(stderr, "invalid field width: %s (8 or 16)\n", optarg);
          std::exit(2);
        }
        break;
      case 1: a.matrix = optarg; break;
      case 2: a.cpu_meta = true; break;
      case 3: a.gpus = to_int(optarg, "GPU count", 1); break;
      case 4: a.slice = to_int(optarg, "slice bytes", 256); streams_given = true; break;
      case 5: a.mul = optarg; break;
      case 6: a.threads = to_int(optarg, "thread count", 0); break;
      case 7: a.op = Args::kMakeConf; break;
      case 8: a.window = to_ll(optarg, "window bytes", 0); break;
      case 9: a.resume = false; break;
      case 10: a.sync = false; break;
      case 12: a.zero_copy = 1; break;
      case 13: a.zero_copy = 0; break;
      case 11: {
        std::string list = optarg ? optarg : "";
        size_t pos = 0;
        while (pos <= list.size()) {
          const size_t comma = list.find(',', pos);
          const std::string item = list.substr(pos, comma == std::string::npos ? std::string::npos : comma - pos);
          a.devices.push_back(to_int(item.c_str(), "device index", 0));
          if (comma == std::string::npos) break;
          pos = comma + 1;
        }
        break;
      }
      case 'h': default: usage(argv[0], gpu); std::exit(c == 'h' ? 0 : 2);
    }
  }
  if (a.zero_copy < 0) a.zero_copy = streams_given ? 0 : 1;
  if (a.op == Args::kEncode) {
    const int cap = a.field_w == 16 ? 65535 : 256;
    if (a.k <= 0 || a.n <= a.k - 1 || a.in_file.empty() || a.n > cap) {
      std::fprintf(stderr, "encode needs -k K -n N -e FILE with 1 <= K <= N <= %d\n", cap);
      std::exit(2);
    }
    if (a.field_w == 16 && a.cpu_meta) {
      std::fprintf(stderr, "-w 16 writes the versioned METADATA (no --cpu-meta form)\n");
      std::exit(2);
    }
  } else if (a.op == Args::kDecode) {
    if (a.in_file.empty() || a.conf.empty()) {
      std::fprintf(stderr, "decode needs -d -i FILE -c CONF\n");
      std::exit(2);
    }
  } else if (a.op == Args::kMakeConf) {
    if (a.k <= 0 || a.n < a.k || a.in_file.empty()) {
      std::fprintf(stderr, "--make-conf needs -k K -n N -e FILE\n");
      std::exit(2);
    }
  } else {
    usage(argv[0], gpu);
    std::exit(2);
  }
  return a;
}

}  // namespace gfrs_cli
