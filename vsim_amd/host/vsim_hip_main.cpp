// vsim_amd/host/vsim_hip_main.cpp — `vsim-hip`, the CLI of the MI355X path.
//
// Same argv and stdout protocol as the reference binary (vsim.cpp:952-1018 main,
// vsim.cpp:749-910 main_gptneox; flags utils.cpp:12-51; sampler utils.cpp:339-422), so
// cformers/interface.py can spawn it unchanged: banner lines, "<|BEGIN> ", " %d " per id
// (prompt echoed in n_batch+1 chunks, then sampled ids), " <END|>"; --return_logits
// prints "logits: %.8f ..." rows.  The model runs in libvsim_hip.so (device resident);
// this file is host control only.  Extra flags: --device N, --mode exact|fast,
// --n_ctx N (reference: fixed 512, vsim.cpp:758), --no-graph.
#include <algorithm>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>
#include <string>
#include <thread>
#include <vector>

#include "../../include/vsim_hip.h"

namespace {

struct Params {
  int32_t seed = -1;
  int32_t n_threads = std::min(4, (int32_t)std::thread::hardware_concurrency());
  int32_t n_predict = 128;
  int32_t repeat_last_n = 64;
  int32_t top_k = 40;
  float top_p = 0.95f;
  float temp = 0.80f;
  float repeat_penalty = 1.30f;
  int32_t n_batch = 8;
  std::string model = "models/lamma-7B/ggml-model.bin";
  std::string prompt;
  bool return_logits = false;
  int device = 0;
  int mode = VSIM_MODE_EXACT;
  int n_ctx = 512;
  bool graph = true;
};

void usage(const char *argv0, const Params &p) {
  fprintf(stderr, "usage: %s <gptneox|gptj|codegen|bloom> [options]\n\n", argv0);
  fprintf(stderr, "options:\n");
  fprintf(stderr, "  -h, --help            show this help message and exit\n");
  fprintf(stderr, "  -s SEED, --seed SEED  RNG seed (default: -1)\n");
  fprintf(stderr, "  -t N, --threads N     accepted for compatibility (default: %d)\n", p.n_threads);
  fprintf(stderr, "  -p PROMPT, --prompt PROMPT  space-separated token ids\n");
  fprintf(stderr, "  -n N, --n_predict N   number of tokens to predict (default: %d)\n", p.n_predict);
  fprintf(stderr, "  --top_k N / --top_p F / --temp F / --repeat_last_n N / --repeat_penalty F\n");
  fprintf(stderr, "  -b N, --batch_size N  prompt batch size (default: %d)\n", p.n_batch);
  fprintf(stderr, "  -m FNAME, --model FNAME  model path\n");
  fprintf(stderr, "  --return_logits       print the next-token logits after the prompt and exit\n");
  fprintf(stderr, "  --device N            GPU index (default 0)\n");
  fprintf(stderr, "  --mode exact|fast     exact = bit-identical to the reference (default)\n");
  fprintf(stderr, "  --n_ctx N             context length (default 512, as the reference)\n");
  fprintf(stderr, "  --no-graph            launch every kernel eagerly\n");
}

// utils.cpp:12-51 (argv[1] is the model type and is skipped)
bool parse(int argc, char **argv, Params &p) {
  for (int i = 2; i < argc; i++) {
    std::string a = argv[i];
    auto next = [&]() -> const char * {
      if (i + 1 >= argc) {
        fprintf(stderr, "error: missing value for %s\n", a.c_str());
        exit(1);
      }
      return argv[++i];
    };
    if (a == "-s" || a == "--seed") p.seed = std::stoi(next());
    else if (a == "-t" || a == "--threads") p.n_threads = std::stoi(next());
    else if (a == "-p" || a == "--prompt") p.prompt = next();
    else if (a == "-n" || a == "--n_predict") p.n_predict = std::stoi(next());
    else if (a == "--top_k") p.top_k = std::stoi(next());
    else if (a == "--top_p") p.top_p = std::stof(next());
    else if (a == "--temp") p.temp = std::stof(next());
    else if (a == "--repeat_last_n") p.repeat_last_n = std::stoi(next());
    else if (a == "--repeat_penalty") p.repeat_penalty = std::stof(next());
    else if (a == "-b" || a == "--batch_size") p.n_batch = std::stoi(next());
    else if (a == "-m" || a == "--model") p.model = next();
    else if (a == "--return_logits") p.return_logits = true;
    else if (a == "--device") p.device = std::stoi(next());
    else if (a == "--mode") p.mode = std::string(next()) == "fast" ? VSIM_MODE_FAST : VSIM_MODE_EXACT;
    else if (a == "--n_ctx") p.n_ctx = std::stoi(next());
    else if (a == "--no-graph") p.graph = false;
    else if (a == "-h" || a == "--help") { usage(argv[0], p); exit(0); }
    else {
      fprintf(stderr, "error: unknown argument: %s\n", a.c_str());
      usage(argv[0], p);
      exit(0);
    }
  }
  return true;
}

// utils.cpp:285-305: the prompt is a list of ids separated by single spaces
std::vector<int32_t> whitespace_tokenize(const std::string &prompt) {
  std::vector<int32_t> t;
  std::string s = prompt;
  while (!s.empty()) {
    auto sp = s.find(' ');
    if (sp == std::string::npos) { t.push_back(std::stoi(s)); break; }
    t.push_back(std::stoi(s.substr(0, sp)));
    s = s.substr(sp + 1);
  }
  return t;
}

// utils.cpp:339-422 sample_top_p_top_k_repeat_penalty
int32_t sample(const float *logits, int n_logits, std::vector<int32_t> &last_n, double repeat_penalty, int top_k,
               double top_p, double temp, std::mt19937 &rng) {
  std::vector<std::pair<double, int32_t>> cand;
  cand.reserve(n_logits);
  const double scale = 1.0 / temp;
  for (int i = 0; i < n_logits; ++i) {
    if (std::find(last_n.begin(), last_n.end(), i) != last_n.end())
      cand.push_back({logits[i] < 0.0 ? logits[i] * scale * repeat_penalty : logits[i] * scale / repeat_penalty, i});
    else
      cand.push_back({logits[i] * scale, i});
  }
  std::partial_sort(cand.begin(), cand.begin() + top_k, cand.end(),
                    [](const std::pair<double, int32_t> &a, const std::pair<double, int32_t> &b) {
                      return a.first > b.first;
                    });
  cand.resize(top_k);
  double maxl = -INFINITY;
  for (auto &kv : cand) maxl = std::max(maxl, kv.first);
  std::vector<double> probs;
  probs.reserve(cand.size());
  double sum = 0.0;
  for (auto &kv : cand) {
    const double pr = std::exp(kv.first - maxl);
    probs.push_back(pr);
    sum += pr;
  }
  for (auto &pr : probs) pr /= sum;
  if (top_p < 1.0f) {
    double cum = 0.0f;
    for (int i = 0; i < (int)probs.size(); i++) {
      cum += probs[i];
      if (cum >= top_p) {
        probs.resize(i + 1);
        cand.resize(i + 1);
        break;
      }
    }
    cum = 1.0 / cum;
    for (auto &pr : probs) pr *= cum;
  }
  std::discrete_distribution<> dist(probs.begin(), probs.end());
  return cand[dist(rng)].second;
}

double now_s() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}

void print_logits(const std::vector<float> &lg, bool end) {
  printf("logits: ");
  for (float v : lg) printf("%.8f ", v);
  printf(end ? " <END|>\n" : "\n");
}

// the per-kernel table of a VSIM_PROFILE=1 run: device ms, share of the device time, launches,
// average time per launch and algorithmic GB/s (Q4_0 weights at 0.625 B/weight, KV rows)
void print_kernel_table(vsim_model *model) {
  struct Row {
    std::string name;
    double ms, bytes;
    long n;
  };
  std::vector<Row> rows;
  char name[128];
  double ms = 0.0, bytes = 0.0, tot = 0.0;
  long n = 0;
  for (int i = 0; vsim_model_profile_kernel(model, i, name, sizeof name, &ms, &n, &bytes) == VSIM_OK; ++i) {
    rows.push_back({name, ms, bytes, n});
    tot += ms;
  }
  printf("%-54s: %10s %7s %8s %10s %9s\n", "device time per kernel (VSIM_PROFILE=1)", "ms", "share", "launches",
         "us/launch", "GB/s");
  for (const Row &r : rows)
    printf("%-54s: %10.3f %6.1f%% %8ld %10.2f %9.1f\n", r.name.c_str(), r.ms, tot > 0 ? 100.0 * r.ms / tot : 0.0, r.n,
           r.n ? 1e3 * r.ms / r.n : 0.0, r.ms > 0 ? r.bytes / (r.ms * 1e6) : 0.0);
  printf("%-54s: %10.3f %6.1f%%\n", "COMPUTE (sum)", tot, 100.0);
}

int run(const Params &params, int arch) {
  const double t_start = now_s();
  std::mt19937 rng(params.seed);
  vsim_model *model = nullptr;
  printf("%s: loading model from '%s' - please wait ...\n", __func__, params.model.c_str());
  if (vsim_model_load_file(params.model.c_str(), arch, params.n_ctx, params.device, 0, -1, &model) != VSIM_OK) {
    fprintf(stderr, "%s: failed to load model from '%s': %s\n", __func__, params.model.c_str(), vsim_last_error());
    return 1;
  }
  vsim_model_set_mode(model, params.mode);
  vsim_model_set_graph(model, params.graph ? 1 : 0);
  // VSIM_PROFILE=1: per-kernel device time at the end of the run, the device counterpart of
  // the reference's per-op time table (monitor.c:196-262, show_time_sep); the steps then run
  // without their hipGraph, one event pair per launch
  const bool profile = getenv("VSIM_PROFILE") && atoi(getenv("VSIM_PROFILE")) != 0;
  if (profile) vsim_model_set_profile(model, 1);
  vsim_hparams hp;
  int n_ctx = 0;
  vsim_model_hparams(model, &hp, &n_ctx, nullptr, nullptr);
  printf("%s: n_vocab = %d\n%s: n_ctx   = %d\n%s: n_embd  = %d\n%s: n_head  = %d\n%s: n_layer = %d\n%s: n_rot   = %d\n",
         __func__, hp.n_vocab, __func__, n_ctx, __func__, hp.n_embd, __func__, hp.n_head, __func__, hp.n_layer,
         __func__, hp.n_rot);
  const double t_load = now_s() - t_start;

  std::vector<int32_t> embd_inp = whitespace_tokenize(params.prompt);
  int n_predict = std::min(params.n_predict, n_ctx - (int)embd_inp.size());
  printf("\n%s: prompt: '%s'\n%s: number of tokens in prompt = %zu\n\n", __func__, params.prompt.c_str(), __func__,
         embd_inp.size());
  printf("sampling parameters: temp = %f, top_k = %d, top_p = %f, repeat_last_n = %i, repeat_penalty = %f\n\n",
         params.temp, params.top_k, params.top_p, params.repeat_last_n, params.repeat_penalty);

  std::vector<float> logits(hp.n_vocab);
  const int32_t warm[5] = {1, 2, 3, 4, 5};
  if (!embd_inp.empty() && (int)embd_inp.size() <= n_ctx &&
      vsim_model_reserve(model, (int)embd_inp.size()) != VSIM_OK) {
    fprintf(stderr, "reserve failed: %s\n", vsim_last_error());
    return 1;
  }
  if (vsim_model_eval(model, 0, warm, 5, nullptr, nullptr, logits.data()) != VSIM_OK) {
    fprintf(stderr, "warm-up eval failed: %s\n", vsim_last_error());
    return 1;
  }
  std::vector<int32_t> last_n(params.repeat_last_n, 0);
  std::vector<int32_t> embd;
  int n_past = 0;
  double t_predict = 0.0, t_sample = 0.0;
  int n_evals = 0, n_decode = 0;
  printf(" embd.size()=%d embd_inp.size()=%d params.n_predict=%d", (int)embd.size(), (int)embd_inp.size(), n_predict);
  printf("\n<|BEGIN> ");
  for (int i = (int)embd.size(); i < (int)embd_inp.size() + n_predict; i++) {
    if (!embd.empty()) {
      const double t0 = now_s();
      if (vsim_model_eval(model, n_past, embd.data(), (int)embd.size(), nullptr, nullptr, logits.data()) != VSIM_OK) {
        printf("Failed to predict\n");
        fprintf(stderr, "%s\n", vsim_last_error());
        return 1;
      }
      t_predict += now_s() - t0;
      ++n_evals;
      if (embd.size() == 1) ++n_decode;
    }
    n_past += (int)embd.size();
    embd.clear();
    if (i >= (int)embd_inp.size()) {
      if (params.return_logits) {
        print_logits(logits, true);
        fflush(stdout);
        vsim_model_free(model);
        return 0;
      }
      const double t0 = now_s();
      const int32_t id = sample(logits.data(), hp.n_vocab, last_n, params.repeat_penalty,
                                (int)(float)params.top_k, params.top_p, params.temp, rng);
      last_n.erase(last_n.begin());
      last_n.push_back(id);
      embd.push_back(id);
      t_sample += now_s() - t0;
    } else {
      for (int k = i; k < (int)embd_inp.size(); k++) {
        if (params.return_logits) print_logits(logits, false);
        embd.push_back(embd_inp[k]);
        last_n.erase(last_n.begin());
        last_n.push_back(embd_inp[k]);
        if ((int)embd.size() > params.n_batch) break;
      }
      i += (int)embd.size() - 1;
    }
    for (auto id : embd)
      if (!params.return_logits) printf(" %d ", id);
    fflush(stdout);
    if (embd.back() == 2) break;
  }
  printf(" <END|>\n");
  printf("\nvsim-hip: load %.3f s, %d evals in %.3f s (%d single-token, %.2f ms/eval), sample %.3f s, total %.3f s\n",
         t_load, n_evals, t_predict, n_decode, n_evals ? 1e3 * t_predict / n_evals : 0.0, t_sample, now_s() - t_start);
  if (profile) print_kernel_table(model);
  vsim_model_free(model);
  return 0;
}

}  // namespace

int main(int argc, char **argv) {
  Params params;
  for (int i = 0; i < argc; i++) printf("argv[%d] = %s\n", i, argv[i]);
  if (argc < 2) { usage(argv[0], params); return 1; }
  parse(argc, argv, params);
  if (params.model.empty() || params.prompt.empty()) return 1;
  if (params.seed < 0) params.seed = (int32_t)time(nullptr);
  printf("%s: seed = %d\n", __func__, params.seed);
  const std::string model_type = argv[1];
  printf("model_type: %s\n", model_type.c_str());
  if (params.return_logits) {
    printf("********************************\n");
    printf("*** return_logits mode ***\n");
    printf("*** setting sampling to greedy ***\n");
    printf("********************************\n");
  }
  if (model_type == "gptneox") return run(params, VSIM_ARCH_GPTNEOX);
  if (model_type == "gptj" || model_type == "codegen") return run(params, VSIM_ARCH_GPTJ);
  if (model_type == "bloom") return run(params, VSIM_ARCH_BLOOM);  // interface.py:92-128 maps BLOOM here
  printf("Unknown model type: %s\n", model_type.c_str());
  return 1;
}
