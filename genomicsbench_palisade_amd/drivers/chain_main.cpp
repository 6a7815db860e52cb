// chain_main.cpp -- CLI drop-in for the chain kernel driver
// (tools/minimap2-acceleration/kernel/scalar/src/main.cpp; benchmarks/chain/src/main.cpp):
//   chain -i <input anchors> -o <output> [-t threads]
// read_call / print_return formats of host_data_io.cpp:13-61 (restated); the kernel is
// host_chain_kernel from libgb_chain_dropin.so (MI355X). Prints "Time in kernel: %.3f sec".
#include <getopt.h>
#include <sys/time.h>

#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../include/gb_compat/minimap2_chain.h"

static void skip_to_eor(FILE *fp) {
  const char *loc = "EOR";
  int ch;
  while (*loc != '\0' && (ch = fgetc(fp)) != EOF)
    if (ch == *loc) loc++;
}

static call_t read_call(FILE *fp) {
  call_t call;
  long long n;
  float avg_qspan;
  int max_dist_x, max_dist_y, bw, n_segs;
  if (fscanf(fp, "%lld%f%d%d%d%d", &n, &avg_qspan, &max_dist_x, &max_dist_y, &bw, &n_segs) != 6) {
    call.n = ANCHOR_NULL;
    call.avg_qspan = .0;
    return call;
  }
  call.n = n;
  call.avg_qspan = avg_qspan;
  call.max_dist_x = max_dist_x;
  call.max_dist_y = max_dist_y;
  call.bw = bw;
  call.n_segs = n_segs;
  call.anchors.resize((size_t)n);
  for (long long i = 0; i < n; i++) {
    unsigned long long x = 0, y = 0;
    if (fscanf(fp, "%llu%llu", &x, &y) != 2) break;
    call.anchors[i].x = x;
    call.anchors[i].y = y;
  }
  skip_to_eor(fp);
  return call;
}

static void print_return(FILE *fp, const return_t &r) {
  fprintf(fp, "%lld\n", (long long)r.n);
  for (anchor_idx_t i = 0; i < r.n; i++) fprintf(fp, "%d\t%d\n", (int)r.scores[i], (int)r.parents[i]);
  fprintf(fp, "EOR\n");
}

int main(int argc, char **argv) {
  std::string in_name, out_name;
  int threads = 1, opt;
  while ((opt = getopt(argc, argv, ":i:o:t:h")) != -1) {
    switch (opt) {
      case 'i': in_name = optarg; break;
      case 'o': out_name = optarg; break;
      case 't': threads = atoi(optarg); break;
      default:
        fprintf(stderr, "usage: chain -i <input file> -o <output file> [-t threads]\n");
        return opt == 'h' ? 0 : 1;
    }
  }
  if (in_name.empty() || out_name.empty()) {
    fprintf(stderr, "usage: chain -i <input file> -o <output file> [-t threads]\n");
    return 1;
  }
  fprintf(stderr, "Input file: %s\n", in_name.c_str());
  fprintf(stderr, "Output file: %s\n", out_name.c_str());
  FILE *in = fopen(in_name.c_str(), "r");
  if (!in) {
    fprintf(stderr, "cannot open %s\n", in_name.c_str());
    return 1;
  }
  FILE *out = fopen(out_name.c_str(), "w");
  if (!out) {
    fprintf(stderr, "cannot open %s\n", out_name.c_str());
    return 1;
  }
  std::vector<call_t> calls;
  std::vector<return_t> rets;
  for (call_t c = read_call(in); c.n != ANCHOR_NULL; c = read_call(in)) calls.push_back(c);
  rets.resize(calls.size());
  struct timeval t0, t1;
  gettimeofday(&t0, nullptr);
  host_chain_kernel(calls, rets, threads);
  gettimeofday(&t1, nullptr);
  const double us = (t1.tv_sec - t0.tv_sec) * 1e6 + (t1.tv_usec - t0.tv_usec);
  for (const auto &r : rets) print_return(out, r);
  // the reference prints %.2f (main.cpp:91); three decimals here (the MI355X call is milliseconds)
  fprintf(stderr, "Time in kernel: %.3f sec\n", us * 1e-6);
  fclose(in);
  fclose(out);
  return 0;
}
