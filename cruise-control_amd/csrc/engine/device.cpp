// Device tables, staging and launch protocol (see device.h).
#include "device.h"
#include "intra.h"
#include "hostpool.h"
#include "prof.h"
#include "threadpin.h"

#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <atomic>
#include <stdexcept>

#include <atomic>
#include <chrono>
#include <mutex>
#include <optional>

#include <pthread.h>
#include <sched.h>

#include <cctype>
#include <fstream>
#include <string>

namespace ccmi {

#define ST ((hipStream_t)st_)
#define EV0 ((hipEvent_t)ev0_)
#define EV1 ((hipEvent_t)ev1_)
#define EV2 ((hipEvent_t)ev2_)

hipError_t launchScanCross(const DevTables& T, const MutTables& M, const UpdateList& U, const DevProgram& prog,
                           const RowRef* reps, const int32_t* cands, int K, int Nr, int N, int c0,
                           unsigned long long* result, unsigned int* done, unsigned long long* mail,
                           unsigned long long seq, hipStream_t st);
hipError_t launchScanSwap(const DevTables& T, const DevProgram& prog, const int32_t* srcs, int S, const int32_t* cbOff,
                          const int32_t* cbRep, int M, const SwapLimit& lim, unsigned long long* result, int32_t* rowVisited,
                          unsigned long long* mail, unsigned long long seq, hipStream_t st, hipEvent_t ev0,
                          hipEvent_t ev1);
hipError_t launchScanPairs(const DevTables& T, const MutTables& M, const UpdateList& U, const DevProgram& prog,
                           const RowRef* pr, const int32_t* pb, int n, int keyBase, unsigned long long* result,
                           unsigned int* done, unsigned long long* mail, unsigned long long seq, hipStream_t st);
hipError_t launchPrep(const MutTables& M, const UpdateList& U, const int4* req, int4* dReq, int nReq4,
                      unsigned long long* result, unsigned int* done, hipStream_t st);
uint32_t scanXcdSliceMinCols();
hipError_t launchScanServer(const DevTables& T, const MutTables& M, const ChainTables& C, const ServerCmd* cmd,
                            const char* pay, const RowRef* pool, unsigned long long* result, unsigned int* done,
                            unsigned long long* mail, unsigned long long* t0, unsigned long long* bell,
                            unsigned long long startSeq, int blocks, hipStream_t st);
hipError_t launchChainPairs(const DevTables& T, const ChainTables& C, const DevProgram& prog, const RowRef* pr,
                            const int32_t* pb, const int32_t* next, int n, int maxAccepts, int32_t* log,
                            ChainResultDev* out, hipStream_t st);
hipError_t launchChainRackRows(const DevTables& T, const ChainTables& C, const DevProgram& prog, const int32_t* rows,
                               int n, const int32_t* cands, int N, int32_t* log, ChainResultDev* out, hipStream_t st);
hipError_t launchSyncLoads(const ChainTables& C, const LoadRow* lrows, int nl, const SlotRow* srows, int ns,
                           hipStream_t st);
hipError_t launchRackRowsGroups(const DevTables& T, const DevProgram& prog, const int32_t* rows, const int32_t* order,
                                const int32_t* gOff, int G, const int32_t* cands, int N, int32_t* res,
                                unsigned long long* evaluated, hipStream_t st);
hipError_t launchStats(const StatsParams& P, const int32_t* tc, const int32_t* topicNrep, const BrokerRec* brokers,
                       const uint8_t* allowedAlive, TopicPartial* scratch, void* partials, StatsOut* out, int ldB,
                       hipStream_t st,
                       hipEvent_t evTopic0, hipEvent_t evTopic1);

hipError_t launchIntra(const IntraArgs& A, hipStream_t st);
hipError_t launchIntraSort(const IntraArgs& A, hipStream_t st);
hipError_t launchIntraCompact(const int32_t* brokers, int n, const int64_t* logOff, const int32_t* count,
                              const int64_t* cOff, const int32_t* rep, const int32_t* src, const int32_t* dst,
                              int32_t* cRep, int32_t* cSrc, int32_t* cDst, hipStream_t st);
hipError_t launchStatsDisks(const int32_t* bDiskOff, const int32_t* bDisks, const double* dCap, const uint8_t* dAlive,
                            const double* dUtil, const uint8_t* bAlive, int B, double balance, DiskStatsOut* out,
                            hipStream_t st);

static void hipCheck(hipError_t e, const char* what) {
  if (e != hipSuccess) throw std::runtime_error(std::string("HIP error in ") + what + ": " + hipGetErrorString(e));
}

template <class T>
static void dalloc(T** p, size_t n) {
  hipCheck(hipMalloc((void**)p, (n ? n : 1) * sizeof(T)), "hipMalloc");
}

static size_t align16(size_t x) { return (x + 15) & ~(size_t)15; }

// HIP's current device is per host thread and starts at 0; a session may run on a thread other than the one that
// created it (the reference's precompute pool, bench.py --requests-per-gpu). Every public entry point that touches
// the device makes the session's ordinal current for its duration and restores the caller's device afterwards.
struct DeviceGuard {
  int prev = -1;
  explicit DeviceGuard(int ordinal) {
    hipCheck(hipGetDevice(&prev), "hipGetDevice");
    if (prev != ordinal) hipCheck(hipSetDevice(ordinal), "hipSetDevice");
    else prev = -1;
  }
  ~DeviceGuard() {
    if (prev >= 0) (void)hipSetDevice(prev);
  }
};

bool deviceLocalCpuList(int ordinal, std::string& out) {
  char bus[64] = {0};
  if (hipDeviceGetPCIBusId(bus, (int)sizeof(bus), ordinal) != hipSuccess) return false;
  for (char* p = bus; *p; ++p) *p = (char)std::tolower((unsigned char)*p);
  std::ifstream f(std::string("/sys/bus/pci/devices/") + bus + "/local_cpulist");
  return (bool)std::getline(f, out);
}

int Device::countGfx950() {
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) return 0;
  int k = 0;
  for (int i = 0; i < n; ++i) {
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, i) == hipSuccess && std::strncmp(prop.gcnArchName, "gfx950", 6) == 0) ++k;
  }
  return k;
}

Device::Device(int ordinal, int B, int R, int P, int T, int maxGoalSlots)
    : ordinal_(ordinal), B_(B), R_(R), P_(P), T_(T), ldB_((B + 3) & ~3), G_(maxGoalSlots) {
  int n = 0;
  hipCheck(hipGetDeviceCount(&n), "hipGetDeviceCount");
  if (ordinal < 0 || ordinal >= n) throw std::runtime_error("no HIP device with ordinal " + std::to_string(ordinal));
  hipCheck(hipSetDevice(ordinal), "hipSetDevice");
  hipDeviceProp_t prop;
  hipCheck(hipGetDeviceProperties(&prop, ordinal), "hipGetDeviceProperties");
  if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
    throw std::runtime_error(std::string("libccmi is built for gfx950, device is ") + prop.gcnArchName);
  hipCheck(hipStreamCreateWithFlags((hipStream_t*)&st_, hipStreamNonBlocking), "hipStreamCreate");
  dalloc(&brokers_, (size_t)B);
  dalloc(&replicas_, (size_t)R);
  dalloc(&parts_, (size_t)P);
  hBrokers_.assign(B, BrokerRec{});
  hParts_.assign(P, PartitionRec{});
  allowedHost_.assign(B, 0u);
  dalloc(&allowedAlive_, ldB_);
  dalloc(&topicCount_, (size_t)T * ldB_);
  dalloc(&topicNrep_, T);
  dalloc(&tUpper_, T);
  dalloc(&tLower_, T);
  dalloc(&dResult_, 4);
  dalloc(&dDone_, 4);
  hipCheck(hipMalloc(&topicScratch_, (size_t)(T ? T : 1) * sizeof(TopicPartial)), "hipMalloc");
  hipCheck(hipMalloc(&statsOut_, 1024), "hipMalloc");
  hipCheck(hipMalloc(&statsPart_, (size_t)kStatsPartBlocks * (kStatD * 8 + kStatI * 4 + 8)), "hipMalloc");
  hipCheck(hipMemset(dDone_, 0, 4 * sizeof(unsigned int)), "hipMemset");
  hipCheck(hipMemset(dResult_, 0xff, 2 * sizeof(unsigned long long)), "hipMemset");
  // host-coherent (fine-grained) mapped memory: kernels read the staging area and write the mailbox directly
  // portable: in a shard group another device's scan server may publish into this mailbox (shard_group.h)
  hipCheck(hipHostMalloc((void**)&hResult_, 1024, hipHostMallocMapped | hipHostMallocCoherent | hipHostMallocPortable),
           "hipHostMalloc");
  hipCheck(hipHostGetDevicePointer((void**)&hResultDev_, hResult_, 0), "hipHostGetDevicePointer");
  std::memset(hResult_, 0, 1024);
  ensureStage(1 << 20);
  ensureReq(1 << 20);
  if (std::getenv("CCMI_STAMPS")) {
    dalloc(&stamps_, 1024 * 8 + 128);  // + the scan server's phase sums at [8192, 8320)
    hipCheck(hipMemset(stamps_, 0, (1024 * 8 + 128) * sizeof(unsigned long long)), "hipMemset");
  }
  hipCheck(hipEventCreate((hipEvent_t*)&ev0_), "hipEventCreate");
  hipCheck(hipEventCreate((hipEvent_t*)&ev1_), "hipEventCreate");
  hipCheck(hipEventCreate((hipEvent_t*)&ev2_), "hipEventCreate");
  hipCheck(hipEventCreate((hipEvent_t*)&evS0_), "hipEventCreate");
  hipCheck(hipEventCreate((hipEvent_t*)&evS1_), "hipEventCreate");
  {  // scan server: on unless CCMI_SERVER=0; CCMI_SERVER_BLOCKS sets its workgroups (multiple of 8, <= 512)
    const char* e = std::getenv("CCMI_SERVER");
    serverUsable_ = !(e && e[0] == '0');
    const char* nb = std::getenv("CCMI_SERVER_BLOCKS");
    if (nb) serverBlocksCap_ = std::max(8, std::min(512, (int)std::strtol(nb, nullptr, 10) / 8 * 8));
    // one workgroup per CU at most, so every workgroup of the server is resident with room for other kernels
    serverBlocksCap_ = std::min(serverBlocksCap_, prop.multiProcessorCount / 8 * 8);
    serverBlocks_ = serverBlocksCap_;
    if (const char* gs = std::getenv("CCMI_GOAL_SPLIT")) goalSplitMax_ = (int)std::strtol(gs, nullptr, 10);
    if (const char* sa = std::getenv("CCMI_SERVER_APPLY")) applyViaServer_ = sa[0] != '0';
    if (const char* gw = std::getenv("CCMI_GOAL_SPLIT_WGS")) goalSplitWgs_ = (int)std::strtol(gw, nullptr, 10);
    if (const char* sw = std::getenv("CCMI_SCAN_WIDTH")) adaptiveWidth_ = std::strcmp(sw, "full") != 0;
    if (const char* ws = std::getenv("CCMI_WG_GOAL_SPLIT")) wgGoalSplit_ = ws[0] != '0';
    if (const char* qs = std::getenv("CCMI_QUERY_SPINS")) spinsBeforeQuery_ = std::strtoull(qs, nullptr, 10);
    if (const char* sm = std::getenv("CCMI_SERVER_STUCK_MS"))
      stuckTicks_ = (unsigned long long)std::max(1.0, std::atof(sm)) * 100000ull;  // 100 MHz s_memrealtime
    if (const char* pk = std::getenv("CCMI_GROUP_PARK_US"))
      parkTicks_ = (unsigned long long)std::max(1.0, std::atof(pk)) * 100ull;
    if (const char* cd = std::getenv("CCMI_CHAIN_DELAY_US"))
      chainDelayTicks_ = (unsigned long long)std::max(0.0, std::atof(cd)) * 100ull;
    if (serverBlocks_ < 8) serverUsable_ = false;
    if (serverUsable_) {
      dalloc(&dServerT0_, 16);  // [0] busy-time stamp, [4, 8) shared-goal pair masks, [8] the doorbell (a line of its own),
                                // [12] the last published seq
      try {
        ensureFg(1 << 20);
        // snapshot pool: 16M rows (256 MB), host-written like the command block. A C2 proposal uploads ~10.6M rows
        // of snapshots; every wrap restarts the server and re-sets the whole queue directory (4M rows wrapped 2-3
        // times per proposal). CCMI_SNAPSHOT_POOL_ROWS sizes it (tests: a small pool wraps often).
        segCap_ = (size_t)16 << 20;
        if (const char* pr = std::getenv("CCMI_SNAPSHOT_POOL_ROWS"))
          segCap_ = (size_t)std::max(1024ll, std::atoll(pr)) & ~(size_t)7;
        hipCheck(hipExtMallocWithFlags((void**)&segPool_, segCap_ * sizeof(RowRef), hipDeviceMallocFinegrained),
                 "hipExtMallocWithFlags snapshot pool");
      } catch (std::exception&) {
        serverUsable_ = false;  // no host-writable fine-grained VRAM: a launch per scan
      }
    }
  }
}

Device::~Device() {
  (void)hipSetDevice(ordinal_);
  try {
    stopServer();
  } catch (std::exception&) {
  }
  if (ST) (void)hipStreamSynchronize(ST);
  if (stamps_) {  // average in-launch phase times of the last 1024 cross/pair scans (workgroup 0)
    std::vector<unsigned long long> h(1024 * 8 + 128);
    if (hipMemcpy(h.data(), stamps_, h.size() * 8, hipMemcpyDeviceToHost) == hipSuccess) {
      if (h[8192])
        std::fprintf(stderr, "[ccmi server stamps] %llu scan commands: copy+acquire %.2f us, stage %.2f us, first tile "
                             "%.2f us, rest to arrival %.2f us (workgroup 0)\n",
                     h[8192], h[8193] * 0.01 / h[8192], h[8194] * 0.01 / h[8192], h[8195] * 0.01 / h[8192],
                     h[8196] * 0.01 / h[8192]);
      if (h[8198])
        std::fprintf(stderr, "[ccmi server stamps] %llu cross/segment commands: request + staging + view loads %.2f us "
                             "of the first tile\n",
                     h[8198], h[8197] * 0.01 / h[8198]);
      if (h[8210])
        std::fprintf(stderr, "[ccmi queue stamps] %llu queue commands: seen -> ready %.2f us, directory batch %.2f us, "
                             "first tile %.2f us, rest to arrival %.2f us, %.2f tiles (workgroup 0)\n",
                     h[8210], h[8211] * 0.01 / h[8210], h[8212] * 0.01 / h[8210], h[8213] * 0.01 / h[8210],
                     h[8214] * 0.01 / h[8210], (double)h[8215] / h[8210]);
      {
        static const char* ops[6] = {"cross", "pairs", "-", "segs", "-", "queue"};
        for (int o = 0; o < 6; ++o)
          if (h[8220 + o])
            std::fprintf(stderr, "[ccmi evaluated] %s: %llu pairs evaluated by the server's tiles\n", ops[o], h[8220 + o]);
      }
      if (h[8230])
        std::fprintf(stderr, "[ccmi chain command stamps] %llu chain commands: seen -> chain start %.2f us (ready -> "
                             "start %.2f us), chain %.2f us, release %.2f us (workgroup 0)\n",
                     h[8230], h[8234] * 0.01 / h[8230], h[8231] * 0.01 / h[8230], h[8232] * 0.01 / h[8230],
                     h[8233] * 0.01 / h[8230]);
      if (h[8200])
        std::fprintf(stderr, "[ccmi chain stamps] %llu chain_pairs launches, %llu accepts: %.2f us per launch in "
                             "evaluation, %.2f us applying, %.2f us in total (thread 0)\n",
                     h[8200], h[8201], h[8202] * 0.01 / h[8200], h[8203] * 0.01 / h[8200], h[8204] * 0.01 / h[8200]);
      if (h[8236] || h[8238])
        std::fprintf(stderr, "[ccmi row stamps] %llu scans with rows: busy %.2f us (the row writer arrived last in "
                             "%llu); %llu scans without rows: busy %.2f us\n",
                     h[8236], h[8236] ? h[8237] * 0.01 / h[8236] : 0.0, h[8235], h[8238],
                     h[8238] ? h[8239] * 0.01 / h[8238] : 0.0);
      if (h[8240])
        std::fprintf(stderr, "[ccmi apply stamps] %llu applies: leadership loads %.2f us, step 0 %.2f us, step 1 %.2f us, "
                             "step 2 + end %.2f us; replica lanes %.2f us, end %.2f us (thread 0, summed over all applies "
                             "/ applies)\n",
                     h[8240], h[8241] * 0.01 / h[8240], h[8242] * 0.01 / h[8240], h[8243] * 0.01 / h[8240],
                     h[8244] * 0.01 / h[8240], h[8245] * 0.01 / h[8240], h[8246] * 0.01 / h[8240]);
      for (int o : {8256, 8261})
        if (h[o])
          std::fprintf(stderr, "[ccmi tile stamps] %llu %s commands, first tile: request landed %.2f us, rows staged %.2f us, "
                       "view loads %.2f us, conjunction to the first slot %.2f us (workgroup 0)\n",
                       h[o], o == 8256 ? "pair" : "cross", h[o + 1] * 0.01 / h[o], h[o + 2] * 0.01 / h[o],
                       h[o + 3] * 0.01 / h[o], h[o + 4] * 0.01 / h[o]);
      if (h[8250])
        std::fprintf(stderr, "[ccmi chain eval stamps] %llu tiles: view loads %.2f us, conjunction %.2f us, tile "
                             "reduction %.2f us (thread 0)\n",
                     h[8250], h[8251] * 0.01 / h[8250], h[8252] * 0.01 / h[8250], h[8253] * 0.01 / h[8250]);
      double acc[5] = {0, 0, 0, 0, 0}, loads = 0;
      int n = 0, nl = 0;
      for (int i = 0; i < 1024; ++i) {
        const unsigned long long* t = &h[i * 8];
        if (!t[0] || !t[1] || !t[2] || !t[3] || !t[4] || !t[5] || t[5] < t[0]) continue;
        for (int k = 0; k < 5; ++k) acc[k] += (double)(t[k + 1] - t[k]) * 0.01;  // 100 MHz -> us
        n++;
        if (t[6] > t[1] && t[6] <= t[2]) {  // scan_cross: the view's loads landed at t[6]
          loads += (double)(t[6] - t[1]) * 0.01;
          nl++;
        }
      }
      if (n)
        std::fprintf(stderr, "[ccmi stamps] %d launches: stage %.2f us, loads+predicate %.2f us (loads %.2f us over %d), "
                             "blockMin %.2f us, tail %.2f us, publish %.2f us\n",
                     n, acc[0] / n, acc[1] / n, nl ? loads / nl : 0.0, nl, acc[2] / n, acc[3] / n, acc[4] / n);
    }
    (void)hipFree(stamps_);
  }
  void* ps[] = {brokers_, replicas_, parts_, allowedAlive_, topicCount_, topicNrep_, topicScratch_, statsOut_,
                statsPart_, dReq_, rowVisited_, dResult_, dDone_, dChainReq_, dRackRes_, tUpper_, tLower_, dRLoad_, dBLoad_, dBLnw_, dBPot_, dPOff_, dPSlots_,
                dPLeader_, pIneligOff_, pIneligB_, topicLead_, tMinLead_, tLeadLim_, hostCap_, dHLoad_, dBHost_,
                dHOff_, dHBrk_};
  for (void* p : ps)
    if (p) (void)hipFree(p);
  if (hChainLog_) (void)hipHostFree(hChainLog_);
  if (hChainOut_) (void)hipHostFree(hChainOut_);
  for (void* p : intraAllocs_)
    if (p) (void)hipFree(p);
  if (fg_) (void)hipFree(fg_);
  if (segPool_) (void)hipFree(segPool_);
  if (qdir_) (void)hipFree(qdir_);
  if (dServerT0_) (void)hipFree(dServerT0_);
  if (hStage_) (void)hipHostFree(hStage_);
  if (hResult_) (void)hipHostFree(hResult_);
  if (ev0_) (void)hipEventDestroy(EV0);
  if (ev1_) (void)hipEventDestroy(EV1);
  if (ev2_) (void)hipEventDestroy(EV2);
  if (evS0_) (void)hipEventDestroy((hipEvent_t)evS0_);
  if (evS1_) (void)hipEventDestroy((hipEvent_t)evS1_);
  if (ST) (void)hipStreamDestroy(ST);
}

// Staging is only rewritten after the previous request completed (every request waits for its mailbox), so
// growing it in place is safe.
void Device::ensureStage(size_t bytes) {
  if (bytes <= stageCap_) return;
  size_t cap = stageCap_ ? stageCap_ : (1 << 20);
  while (cap < bytes) cap <<= 1;
  char* fresh = nullptr;
  hipCheck(hipHostMalloc((void**)&fresh, cap, hipHostMallocMapped | hipHostMallocCoherent), "hipHostMalloc stage");
  if (hStage_) {
    std::memcpy(fresh, hStage_, stageUsed_);
    (void)hipHostFree(hStage_);
  }
  hStage_ = fresh;
  hipCheck(hipHostGetDevicePointer((void**)&hStageDev_, hStage_, 0), "hipHostGetDevicePointer");
  stageCap_ = cap;
}

void Device::ensureReq(size_t bytes) {
  if (bytes <= reqCap_) return;
  size_t cap = reqCap_ ? reqCap_ : (1 << 20);
  while (cap < bytes) cap <<= 1;
  if (dReq_) (void)hipFree(dReq_);
  hipCheck(hipMalloc((void**)&dReq_, cap), "hipMalloc request");
  reqCap_ = cap;
}

// ------------------------------------------------------------------------------------------------ scan server
namespace {
constexpr size_t kCmdBytes = 256;  // the ServerCmd block; the payload follows
static_assert(sizeof(ServerCmd) <= kCmdBytes, "ServerCmd fits its block");
// Persistent scan servers of this process per device and their workgroups: a session starts one only while the
// device's total stays within kServerBudget workgroups (one workgroup per CU), so no persistent launch holds the CU
// slots another server's workgroups wait for; a session that finds no room launches per scan. Concurrent calls on a
// device share the budget: a server started while A sessions of the process are inside an optimization call on the
// device gets kServerBudget / A workgroups (servers restart at every goal's statistics, so the shares follow the
// calls), and the sessions' servers run side by side on disjoint CUs instead of one session launching per scan
// behind another's resident server.
constexpr int kServerBudget = 256;
std::mutex g_serverMu;
int g_serverWgs[64] = {};
int g_activeCalls[64] = {};
// the scan server's direct pollers of the command word (DevTables.directPollers)
int directPollers() {
  static const int v =
      std::getenv("CCMI_DIRECT_POLLERS") ? std::max(1, std::min(32, std::atoi(std::getenv("CCMI_DIRECT_POLLERS")))) : 8;
  return v;
}
double nowSeconds() {
  return std::chrono::duration<double>(std::chrono::steady_clock::now().time_since_epoch()).count();
}
inline void hostStoreFence() { __builtin_ia32_sfence(); }
// a launched chain longer than this is reported as stuck (C2's longest chain takes milliseconds)
constexpr double kChainWaitSeconds = 120.0;
}  // namespace

void Device::ensureFg(size_t bytes) {
  if (bytes <= fgCap_) return;
  stopServer();
  size_t cap = fgCap_ ? fgCap_ : (1 << 20);
  while (cap < bytes) cap <<= 1;
  if (fg_) hipCheck(hipFree(fg_), "hipFree fine-grained");
  fg_ = nullptr;
  fgCap_ = 0;
  hipCheck(hipExtMallocWithFlags((void**)&fg_, cap, hipDeviceMallocFinegrained), "hipExtMallocWithFlags fine-grained");
  fgCap_ = cap;
  // the command block starts with sequence 0 = "nothing new" (written through the BAR; never read back by the host)
  ServerCmd z;
  std::memset(&z, 0, sizeof(z));
  z.seq = lastCmdSeq_;
  std::memcpy(fg_, &z, sizeof(z));
  hostStoreFence();
  progSent_ = false;
}

// A shard-group session's server parks (ends its launch) when a group scan waits too long for the other ranks
// (kernels/scan.hip, shard_group.h): its workgroups follow workgroup 0's exit record out, so the stream drains by
// itself; the budget and the timing are settled as for a stop.
void Device::retireParkedServer() {
  if (serverTimed_) (void)hipEventRecord((hipEvent_t)evS1_, ST);
  hipCheck(hipStreamSynchronize(ST), "parked scan server");
  serverOn_ = false;
  {
    std::lock_guard<std::mutex> lk(g_serverMu);
    g_serverWgs[ordinal_ & 63] -= serverBlocks_;
  }
  if (serverTimed_) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, (hipEvent_t)evS0_, (hipEvent_t)evS1_) == hipSuccess) perf.serverResidentMs += ms;
    serverTimed_ = false;
  }
  prof().count(31, "server.parks", 1);
}

// A group session moves mail[7] (the last posted command) forward before each command; false: the server parked
// after its last command instead (it is retired here, nothing of the new command ran).
bool Device::claimServer() {
  if (!grpHost_) return true;
  unsigned long long expect = lastCmdSeq_;
  if (__atomic_compare_exchange_n(&hResult_[7], &expect, seq_ + 1, false, __ATOMIC_ACQ_REL, __ATOMIC_ACQUIRE))
    return true;
  retireParkedServer();
  return false;
}

void Device::stopServer() {
  if (!serverOn_) return;
  DeviceGuard dg(ordinal_);
  if (!claimServer()) return;  // parked: already ended
  ServerCmd* c = (ServerCmd*)fg_;
  *(volatile unsigned long long*)&c->seq = (seq_ + 1) | kSeqBusy;  // seqlock (devtypes.h kSeqBusy)
  hostStoreFence();
  volatile int32_t* op = &c->op;
  *op = SOP_EXIT;
  hostStoreFence();
  lastCmdSeq_ = ++seq_;
  *(volatile unsigned long long*)&c->seq = lastCmdSeq_;
  hostStoreFence();
  serverOn_ = false;
  {
    std::lock_guard<std::mutex> lk(g_serverMu);
    g_serverWgs[ordinal_ & 63] -= serverBlocks_;
  }
  if (serverTimed_) (void)hipEventRecord((hipEvent_t)evS1_, ST);
  hipCheck(hipStreamSynchronize(ST), "scan server exit");
  if (serverTimed_) {
    float ms = 0.f;
    if (hipEventElapsedTime(&ms, (hipEvent_t)evS0_, (hipEvent_t)evS1_) == hipSuccess) perf.serverResidentMs += ms;
    serverTimed_ = false;
  }
}

// A cross / pair scan the running (or a newly started) server can take: its rows fit the LDS overlay and, when the
// program reads topic counts, no topic delta is pending (those are applied by `prep` before any workgroup reads).
// The pending rows for a served scan. A scan whose program reads topic counts cannot be served while topic-count
// deltas are pending (the LDS overlay shadows records, not counts), so those go to the tables first in an apply-only
// server command — a SOP_CHAIN with no pairs: workgroup 0 applies the rows and deltas and releases them — two server
// round trips instead of stopping the server for a prep + scan launch and restarting it (CCMI_SERVER_APPLY=0: off).
Device::Staged Device::packForServer(const DevProgram& prog, bool readsTc, bool& serve) {
  Staged g = packUpdates(0);
  serve = serveScan(prog, g, readsTc);
  if (serve || !readsTc || g.nt == 0 || !applyViaServer_ || !serverUsable_ || !serverAllowed_ || !dRLoad_) return g;
  unpackUpdates(g);
  static const int32_t none = 0;
  if (serverChain(prog, CM_PAIRS, &none, 0, &none, 0, &none, 0, 0, 0, 0)) {
    perf.serverChains--;  // not a chain
    perf.serverApplies++;
  }
  g = packUpdates(0);
  serve = serveScan(prog, g, readsTc);
  return g;
}

bool Device::serveScan(const DevProgram& prog, const Staged& g, bool readsTopicCounts) {
  (void)prog;
  if (!serverUsable_ || !serverAllowed_) return false;
  if (g.nb > kOverlayRows || g.nr > kOverlayRows || g.np > kOverlayRows) return false;
  if (readsTopicCounts && g.nt > 0) return false;
  return true;
}

// Start the server unless it runs (restarting one the host left idle for a while, far from the device's 2 s
// watchdog); false when the device already has its budget of servers (the caller launches instead).
void Device::limitServerBlocks(int blocks) {
  stopServer();
  serverBlocksCap_ = std::max(8, std::min(serverBlocksCap_, blocks / 8 * 8));
  serverBlocks_ = serverBlocksCap_;
}

void Device::callBegin() {
  std::lock_guard<std::mutex> lk(g_serverMu);
  ++g_activeCalls[ordinal_ & 63];
}
void Device::callEnd() {
  std::lock_guard<std::mutex> lk(g_serverMu);
  --g_activeCalls[ordinal_ & 63];
}

bool Device::ensureServer() {
  if (serverOn_ && nowSeconds() - lastServerUse_ > 0.25) stopServer();
  if (serverOn_) {
    // A running server is resized when the device's concurrent calls changed its share: shrunk when another call
    // began (that call's server needs the workgroups this one holds, one workgroup per CU), grown when its share at
    // least doubled. The stop retires the launch between two commands, and the relaunch below takes the new share.
    int target;
    {
      std::lock_guard<std::mutex> lk(g_serverMu);
      const int active = std::max(1, g_activeCalls[ordinal_ & 63]);
      const int want = std::min(serverBlocksCap_, std::max(8, kServerBudget / active / 8 * 8));
      const int room = kServerBudget - g_serverWgs[ordinal_ & 63] + serverBlocks_;  // with this server's returned
      target = std::min(want, room / 8 * 8);
    }
    if (target == serverBlocks_ || (target > serverBlocks_ && target < 2 * serverBlocks_)) return true;
    stopServer();
  }
  progSent_ = false;
  {
    std::lock_guard<std::mutex> lk(g_serverMu);
    const int active = std::max(1, g_activeCalls[ordinal_ & 63]);
    // this call's share of the device's server budget, or what the other calls' servers leave of it (they shrink to
    // their own shares at their next commands)
    const int room = (kServerBudget - g_serverWgs[ordinal_ & 63]) / 8 * 8;
    const int want = std::min({serverBlocksCap_, std::max(8, kServerBudget / active / 8 * 8), room});
    if (want < 8) return false;
    g_serverWgs[ordinal_ & 63] += want;
    serverBlocks_ = want;  // this launch's workgroups (the stop returns them)
  }
  // the arrival counter and the result word start clean for every server launch, whatever an earlier launch left
  hipCheck(hipMemsetAsync(dDone_, 0, sizeof(unsigned int), ST), "reset server arrivals");
  hipCheck(hipMemsetAsync(dResult_, 0xff, sizeof(unsigned long long), ST), "reset server result");
  hipCheck(hipMemsetAsync(dServerT0_ + 8, 0, sizeof(unsigned long long), ST), "reset server doorbell");
  hipCheck(hipMemsetAsync(dServerT0_ + 12, 0, sizeof(unsigned long long), ST), "reset server publication word");
  hipCheck(hipMemsetAsync(dServerT0_ + 4, 0xff, 4 * sizeof(unsigned long long), ST), "reset server mask words");
  __atomic_store_n(&hResult_[7], lastCmdSeq_, __ATOMIC_RELEASE);  // the new launch's last command (parking, groups)
  serverTimed_ = timing;
  if (serverTimed_) (void)hipEventRecord((hipEvent_t)evS0_, ST);
  hipCheck(launchScanServer(tables(), mutTables(), chainTables(), (const ServerCmd*)fg_, fg_ + kCmdBytes, segPool_,
                            dResult_, dDone_, hResultDev_, dServerT0_, dServerT0_ + 8, lastCmdSeq_, serverBlocks_, ST),
           "scan_server");
  serverOn_ = true;
  perf.serverLaunches++;
  perf.scanLaunches++;
  return true;
}

// The program into the payload's program slot when it changed (or the server is new); its version
int Device::serverProgram(const DevProgram& prog, char* pay) {
  if (progSent_ && std::memcmp(&prog, &lastProg_, sizeof(DevProgram)) == 0) return progVer_;
  std::memcpy(pay, &prog, sizeof(DevProgram));
  lastProg_ = prog;
  progSent_ = true;
  perf.serverPayloadBytes += (int64_t)sizeof(DevProgram);
  prof().addPayload((int64_t)sizeof(DevProgram));
  return ++progVer_;
}

// Publish a command (seqlock: the sequence word marked busy, every other field, then behind store fences the new
// sequence word) and wait for its result. false: the server's idle watchdog ended it before it saw the command —
// nothing of the command ran, and the caller takes its launch path.
bool Device::postCommand(ServerCmd& c, bool rowsSent) {
  const bool tp = prof().on && c.op == SOP_CHAIN;  // CCMI_PROFILE: a chain command's busy-record wait and round trip
  const auto tA = tp ? std::chrono::steady_clock::now() : std::chrono::steady_clock::time_point();
  collectServerBusy();
  if (tp)
    prof().count(40, "chain.ns.busywait",
                 (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - tA).count());
  if (!claimServer()) return false;  // parked after its last command: the caller takes its launch path
  c.rowsEpoch = rowsEpoch_;
  std::optional<NsScope> nsHdr;
  if (prof().on) nsHdr.emplace(7, "srv.ns.header");  // CCMI_PROFILE: the header's seqlock writes and fences
  *(volatile unsigned long long*)fg_ = (seq_ + 1) | kSeqBusy;
  hostStoreFence();
  std::memcpy(fg_ + sizeof(unsigned long long), (const char*)&c + sizeof(unsigned long long),
              sizeof(ServerCmd) - sizeof(unsigned long long));
  hostStoreFence();
  lastCmdSeq_ = ++seq_;
  *(volatile unsigned long long*)fg_ = lastCmdSeq_ | (c.nActive >= directPollers() ? kSeqAll : 0ull);
  hostStoreFence();
  nsHdr.reset();
  const auto tW = tp ? std::chrono::steady_clock::now() : std::chrono::steady_clock::time_point();
  const bool seen = waitMail(seq_, true);
  if (tp)
    prof().count(41, "chain.ns.roundtrip",
                 (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - tW).count());
  if (parkedPending_) {  // the result came after the server parked (a slow shard group): retire the ended launch
    parkedPending_ = false;
    retireParkedServer();
  }
  if (!seen) {
    serverOn_ = false;
    {
      std::lock_guard<std::mutex> lk(g_serverMu);
      g_serverWgs[ordinal_ & 63] -= serverBlocks_;
    }
    perf.serverIdleExits++;
    return false;
  }
  if (rowsSent) ++rowsEpoch_;
  lastServerUse_ = nowSeconds();
  busyPending_ = true;  // its busy time lands in mail[5] just after the word (collected before the next command)
  busySeq_ = seq_;
  return true;
}

// The last server command's busy time (mail[5], tagged with its sequence; scan.hip scan_server's publish)
void Device::collectServerBusy() {
  if (!busyPending_) return;
  busyPending_ = false;
  const unsigned long long want = busySeq_ & 0xffffffull;
  volatile unsigned long long* mail = (volatile unsigned long long*)hResult_;
  const double t0 = nowSeconds();
  for (uint64_t spin = 0;; ++spin) {
    const unsigned long long w = __atomic_load_n(&mail[5], __ATOMIC_ACQUIRE);
    if ((w >> 40) == want) {
      perf.serverBusyMs += (double)(w & ((1ull << 40) - 1)) * 1e-5;  // 100 MHz ticks
      return;
    }
    // the store left the device right behind the result word: a miss here is a lost diagnostic, never a wait on work
    if ((spin & 1023) == 1023 && nowSeconds() - t0 > 0.1) return;
  }
}

// params: CROSS {K, Nr, N, c0, sliced, -}; PAIRS {n, keyBase, -, -, -, -}
int64_t Device::serverRun(const DevProgram& prog, const Staged& g, int op, const void* A, size_t nA,
                          const int32_t* C, size_t nC, const int32_t params[6]) {
  // payload: [program | rows | A | C]; the program slot is always reserved so offsets never depend on whether it is
  // resent (a restarted server has no program in LDS: it gets the program again whatever the host sent before)
  const size_t oProg = 0, oRows = align16(sizeof(DevProgram));
  const size_t rows = g.end;  // [broker | replica | partition rows | topic deltas] as packUpdates laid them out
  const size_t aBytes = op == SOP_SEGS ? nA * sizeof(SegEntry) : nA * sizeof(RowRef);
  const size_t oA = oRows + rows, oC = oA + align16(aBytes), end = oC + align16(nC * 4);
  ensureFg(kCmdBytes + end);
  if (!ensureServer()) return INT64_MIN;
  std::optional<NsScope> nsPay;
  if (prof().on) nsPay.emplace(6, "srv.ns.payload");  // CCMI_PROFILE: the payload's writes through the BAR
  char* pay = fg_ + kCmdBytes;
  const int ver = serverProgram(prog, pay + oProg);
  perf.serverPayloadBytes += (int64_t)(rows + aBytes + nC * 4);
  prof().addPayload((int64_t)(rows + aBytes + nC * 4));
  prof().count(11, "srv.bytes.rows", (int64_t)rows);
  prof().count(12, "srv.bytes.A", (int64_t)aBytes);
  prof().count(13, "srv.bytes.C", (int64_t)nC * 4);
  if (rows) std::memcpy(pay + oRows, hStage_, rows);
  if (op == SOP_SEGS) std::memcpy(pay + oA, A, aBytes);
  else if (nA) writeRowRefs(pay + oA, (const int32_t*)A, nA);
  if (nC) std::memcpy(pay + oC, C, nC * 4);
  ServerCmd c;
  std::memset(&c, 0, sizeof(c));
  c.op = op;
  if (op == SOP_CROSS || op == SOP_SEGS) {
    c.K = params[0];
    c.Nr = params[1];
    c.N = params[2];
    c.c0 = params[3];
    c.sliced = params[4];
    c.nSegs = params[5];
  } else {
    c.n = params[0];
    c.keyBase = params[1];
  }
  c.progVer = ver;
  // the scan's site (op, action, goal count, filter: one driver loop of one goal) for its speculative width; sliced
  // scans split columns over the XCDs and keep the full width
  const bool sliced = op != SOP_PAIRS && params[4] != 0;
  const uint64_t site = (uint64_t)op | ((uint64_t)(uint32_t)prog.action << 3) | ((uint64_t)(uint32_t)prog.nGoals << 8) |
                        ((uint64_t)(uint32_t)prog.filter << 16) | ((uint64_t)sliced << 24);
  {  // every tile of the first sweep gets its own workgroup; a smaller scan leaves the others out of the command
    const uint64_t whole = op == SOP_PAIRS ? (uint64_t)params[0] : (uint64_t)params[0] * (uint64_t)params[1];
    uint64_t total = whole;
    if (adaptiveWidth_) {
      // Speculative width: the first sweep covers twice the depth of this site's last winner (plus eight tiles), or
      // everything after a scan without one. Tiles past the winner are evaluated for nothing (their reads are the
      // excess HBM traffic of first-fit scans); a winner beyond the sweep is found by the strided next sweeps, so
      // the first fit is the same either way. A column-sliced scan (every XCD sweeps its own columns of each row)
      // counts its depth in rows: the first sweep covers twice the winner's row plus one of every slice.
      const auto it = lastDepth_.find(site);
      if (it != lastDepth_.end() && it->second >= 0)
        total = std::min<uint64_t>(total, sliced ? (2 * (uint64_t)it->second + 1) * (uint64_t)params[1]
                                                 : 2 * (uint64_t)it->second + 8 * 256);
    }
    auto wgsFor = [&](int parts) {
      const uint64_t tile = 256 / (uint64_t)parts;
      const uint64_t need = (total + tile - 1) / tile;
      return std::max<uint64_t>(8, (need + 7) / 8 * 8);
    };
    // Goal-parallel tiles: when the scan's first sweep fits the server at 2 or 4 waves per candidate, each wave
    // evaluates a share of the goals (the conjunction's latency over the prior goals is most of a small command's
    // in-kernel time, and the workgroups a small command leaves idle take the other shares).
    int parts = 1;
    for (int p : {4, 2})
      if (p <= goalSplitMax_ && p <= prog.nGoals && wgsFor(p) <= (uint64_t)std::min(goalSplitWgs_, serverBlocks_)) {
        parts = p;
        break;
      }
    c.goalParts = parts;
    c.nActive = (int32_t)std::min<uint64_t>(wgsFor(parts), (uint64_t)serverBlocks_);
    // A pair command of at most four tiles of 64: each tile's goals are shared by enough workgroups to leave about one
    // goal per wave (scan.hip, c.wgParts: the conjunction is most of such a command's first tile), and one more
    // workgroup without a tile writes the command's rows
    c.wgParts = 1;
    if (wgGoalSplit_ && op == SOP_PAIRS && parts == 4 && whole <= 4 * 64 && prog.nGoals > parts) {
      const int tiles = (int)((whole + 63) / 64);
      // the sharing workgroups and the writer within the direct pollers, which all see the command at once
      const int share = std::min((prog.nGoals + parts - 1) / parts, (directPollers() - 1) / tiles);
      if (share >= 2 && tiles * share + 1 <= serverBlocks_) {
        c.wgParts = share;
        c.nActive = std::max(c.nActive, tiles * share + 1);
      }
    }
    if (prof().on && op == SOP_PAIRS)  // CCMI_PROFILE: pair-scan sizes
      prof().count(whole <= 64 ? 58 : whole <= 256 ? 59 : whole <= 2048 ? 60 : 61,
                   whole <= 64 ? "pairs.n<=64" : whole <= 256 ? "pairs.n<=256" : whole <= 2048 ? "pairs.n<=2048" : "pairs.n>2048");
  }
  const bool grouped = grpHost_ && combineArmed_ && (op == SOP_CROSS || op == SOP_SEGS || op == SOP_PAIRS);
  if (grouped) {  // the server folds this scan's key into the group's slot; the group's last rank publishes the minimum
    c.combineBlock = grpDev_;
    c.combineSlot = (int32_t)(grpCalls_ & 1);
    c.combineRank = grpRank_;
    c.combineCount = grpCount_;
  }
  c.nb = g.nb;
  c.nr = g.nr;
  c.np = g.np;
  c.nt = g.nt;
  c.oProg = (uint32_t)oProg;
  c.oB = (uint32_t)(oRows + g.obr);
  c.oR = (uint32_t)(oRows + g.orr);
  c.oP = (uint32_t)(oRows + g.opr);
  c.oT = (uint32_t)(oRows + g.otd);
  c.oA = (uint32_t)oA;
  c.oC = (uint32_t)oC;
  nsPay.reset();
  if (!postCommand(c, (g.nb | g.nr | g.np | g.nt) != 0)) return INT64_MIN;
  perf.serverScans++;
  const unsigned long long lo = hResult_[0] & 0xffffffffull;
  const int64_t key = lo == 0 ? -1 : (int64_t)(lo - 1);
  if (grouped) {
    ++grpCalls_;
    devCombined_ = true;
    combineArmed_ = false;
  }
  if (adaptiveWidth_) {  // the winner's position in the first-sweep order (sliced: its row; -1: none)
    int64_t depth = -1;
    if (key >= 0)
      depth = op == SOP_PAIRS ? key - params[1]
              : sliced        ? key / params[2]
                              : (key / params[2]) * params[1] + (key % params[2] - params[3]);
    lastDepth_[site] = depth;
  }
  return key;
}

// A K7 chain as a server command (SOP_CHAIN): payload [program | rows | load rows | slot rows | request]. false: the
// server cannot take it (not usable here, over budget, or ended by its watchdog before it saw the command) — the
// pending rows are back in their lists and the caller launches the chain kernel instead.
bool Device::serverChain(const DevProgram& prog, int mode, const int32_t* a0, int n0, const int32_t* a1, int n1,
                         const int32_t* a2, int n2, int n, int m, int maxAccepts) {
  if (!serverUsable_ || !serverAllowed_ || !dRLoad_) return false;
  const auto tS = prof().on ? std::chrono::steady_clock::now() : std::chrono::steady_clock::time_point();
  const size_t nl = lrows.size(), ns = srows.size();
  lrowsSent_ = nl;
  srowsSent_ = ns;
  // CM_PAIRS: a0 (the pairs' replicas) goes out as RowRefs (scan.hip serverChain's request layout)
  const bool refs = mode == CM_PAIRS;
  const size_t words = (size_t)n0 * (refs ? 4 : 1) + n1 + n2;
  const size_t oRows = align16(sizeof(DevProgram));
  const Staged g = packUpdates(0);
  if (g.nb > kOverlayRows || g.nr > kOverlayRows || g.np > kOverlayRows) {  // the server stages rows in its LDS overlay
    unpackUpdates(g);
    return false;
  }
  const size_t oL = oRows + g.end, oS = oL + align16(nl * sizeof(LoadRow)), oA = oS + align16(ns * sizeof(SlotRow));
  const size_t end = oA + align16(words * 4);
  ensureFg(kCmdBytes + end);
  if (!ensureServer()) {
    unpackUpdates(g);
    return false;
  }
  if (words * 4 > chainReqCap_) {
    if (dChainReq_) hipCheck(hipFree(dChainReq_), "hipFree chain request");
    dChainReq_ = nullptr;
    chainReqCap_ = std::max<size_t>(words * 8, 1 << 16);
    hipCheck(hipMalloc((void**)&dChainReq_, chainReqCap_), "hipMalloc chain request");
  }
  char* pay = fg_ + kCmdBytes;
  const int ver = serverProgram(prog, pay);
  if (g.end) std::memcpy(pay + oRows, hStage_, g.end);
  if (nl) std::memcpy(pay + oL, lrows.data(), nl * sizeof(LoadRow));
  if (ns) std::memcpy(pay + oS, srows.data(), ns * sizeof(SlotRow));
  const size_t a0Bytes = (size_t)n0 * (refs ? sizeof(RowRef) : 4);
  if (refs) writeRowRefs(pay + oA, a0, (size_t)n0);
  else std::memcpy(pay + oA, a0, a0Bytes);
  if (n1) std::memcpy(pay + oA + a0Bytes, a1, (size_t)n1 * 4);
  if (n2) std::memcpy(pay + oA + a0Bytes + (size_t)n1 * 4, a2, (size_t)n2 * 4);
  perf.serverPayloadBytes += (int64_t)(end - oRows);
  prof().addPayload((int64_t)(end - oRows));
  ServerCmd c;
  std::memset(&c, 0, sizeof(c));
  c.op = SOP_CHAIN;
  c.progVer = ver;
  c.nActive = 1;
  c.nb = g.nb;
  c.nr = g.nr;
  c.np = g.np;
  c.nt = g.nt;
  c.oProg = 0;
  c.oB = (uint32_t)(oRows + g.obr);
  c.oR = (uint32_t)(oRows + g.orr);
  c.oP = (uint32_t)(oRows + g.opr);
  c.oT = (uint32_t)(oRows + g.otd);
  c.oA = (uint32_t)oA;
  c.chainMode = mode;
  c.chainN = n;
  c.chainM = m;
  c.maxAccepts = maxAccepts;
  c.nl = (int32_t)nl;
  c.ns = (int32_t)ns;
  c.oL = (uint32_t)oL;
  c.oS = (uint32_t)oS;
  c.chainReq = (unsigned long long)(uintptr_t)dChainReq_;
  c.chainLog = (unsigned long long)(uintptr_t)hChainLogDev_;
  c.chainOut = (unsigned long long)(uintptr_t)hChainOutDev_;
  // a chain writes the tables: every later command's workgroups acquire before reading them
  const auto tP = prof().on ? std::chrono::steady_clock::now() : std::chrono::steady_clock::time_point();
  if (prof().on) prof().count(39, "chain.ns.stage", (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(tP - tS).count());
  if (!postCommand(c, true)) {
    unpackUpdates(g);
    return false;
  }
  lrows.clear();
  srows.clear();
  perf.serverChains++;
  return true;
}

// A launched kernel's completion on the session stream, bounded: past `seconds` the wait reports what it waited for and
// the mailbox / server state instead of blocking forever.
void Device::streamWait(const char* what, double seconds) {
  const double t0 = nowSeconds();
  for (uint64_t spins = 0;; ++spins) {
    const hipError_t q = hipStreamQuery(ST);
    if (q == hipSuccess) return;
    if (q != hipErrorNotReady) hipCheck(q, what);
    if (nowSeconds() - t0 > seconds) {
      char msg[256];
      std::snprintf(msg, sizeof(msg), "%s did not complete within %.0f s (server %s, mail %016llx, server exit %016llx)",
                    what, seconds, serverOn_ ? "on" : "off", (unsigned long long)hResult_[0],
                    (unsigned long long)hResult_[3]);
      throw std::runtime_error(msg);
    }
    if (spins < 4096) __builtin_ia32_pause();
    else sched_yield();
  }
}

void Device::writeRowRefs(char* dst, const int32_t* reps, size_t n) const {
  if (!rowBroker_) throw std::runtime_error("scan rows need the model's row source (Device::setRowSource)");
  RowRef buf[64];  // built in cache, then copied out in 1 KB pieces (dst may be write-combined device memory)
  for (size_t i = 0; i < n; i += 64) {
    const size_t m = std::min<size_t>(64, n - i);
    for (size_t k = 0; k < m; ++k) {
      const int r = reps[i + k], p = rowPart_[r];
      buf[k] = RowRef{r, rowBroker_[r], p, partTopic_[p]};
    }
    std::memcpy(dst + i * sizeof(RowRef), buf, m * sizeof(RowRef));
  }
}

DevTables Device::tables() const {
  DevTables t;
  t.brokers = brokers_;
  t.replicas = replicas_;
  t.parts = parts_;
  t.topicCount = topicCount_;
  t.tUpper = tUpper_;
  t.tLower = tLower_;
  t.stamps = stamps_;
  t.pIneligOff = pIneligOff_;
  t.pIneligB = pIneligB_;
  t.topicLead = topicLead_;
  t.tMinLead = tMinLead_;
  t.tLeadLim = tLeadLim_;
  t.hostCap = hostCap_;
  t.B = B_;
  t.R = R_;
  t.P = P_;
  t.ldB = ldB_;
  static const int pollMode = std::getenv("CCMI_SERVER_POLL") ? std::atoi(std::getenv("CCMI_SERVER_POLL")) : 0;
  t.pollMode = pollMode;
  static const int seqRecheck = std::getenv("CCMI_SEQ_RECHECK") ? std::atoi(std::getenv("CCMI_SEQ_RECHECK")) : 0;
  t.seqRecheck = seqRecheck;
  static const int conjRepeat = std::getenv("CCMI_CONJ_REPEAT") ? std::atoi(std::getenv("CCMI_CONJ_REPEAT")) : 0;
  t.conjRepeat = conjRepeat;
  t.directPollers = directPollers();
  t.stuckTicks = stuckTicks_;
  t.parkTicks = parkTicks_;
  t.chainDelayTicks = chainDelayTicks_;
  return t;
}

// Static columns are kept in host copies of the broker / partition records until uploadDynamic packs and
// uploads the whole records (the caller uploads static columns first).
void Device::uploadStatic(const double* bCapRM, const int32_t* rPart, const int32_t* rOrig, const int32_t* pOff,
                          const int32_t* topicNrep, const int32_t* bRack, const int32_t* pTopic) {
  DeviceGuard dg(ordinal_);
  stopServer();
  for (int b = 0; b < B_; ++b) {
    BrokerRec& x = hBrokers_[b];
    for (int k = 0; k < 4; ++k) x.cap[k] = bCapRM[(size_t)k * B_ + b];
    x.rack = bRack[b];
  }
  hRPart_.assign(rPart, rPart + R_);
  hROrig_.assign(rOrig, rOrig + R_);
  hPOff_.assign(pOff, pOff + P_ + 1);
  for (int p = 0; p < P_; ++p) {
    hParts_[p].topic = pTopic[p];
    hParts_[p].n = pOff[p + 1] - pOff[p];
  }
  bRackHost_.assign(bRack, bRack + B_);
  hipCheck(hipMemcpy(topicNrep_, topicNrep, sizeof(int32_t) * T_, hipMemcpyHostToDevice), "upload topicNrep");
}

void Device::uploadIneligible(const int32_t* off, const int32_t* brokers, int n) {
  DeviceGuard dg(ordinal_);
  stopServer();
  if (n <= 0) return;
  hipCheck(hipMalloc((void**)&pIneligOff_, sizeof(int32_t) * (P_ + 1)), "hipMalloc pIneligOff");
  hipCheck(hipMalloc((void**)&pIneligB_, sizeof(int32_t) * n), "hipMalloc pIneligB");
  hipCheck(hipMemcpy(pIneligOff_, off, sizeof(int32_t) * (P_ + 1), hipMemcpyHostToDevice), "upload pIneligOff");
  hipCheck(hipMemcpy(pIneligB_, brokers, sizeof(int32_t) * n, hipMemcpyHostToDevice), "upload pIneligB");
}

void Device::uploadDynamic(const double* bUtilRM, const int32_t* bNrep, const int32_t* bNlead, const double* bPot,
                           const double* bLeadNwIn, const uint8_t* bAlive, const double* rUtilRM,
                           const int32_t* rBroker, const uint8_t* rFlags, const int32_t* pBrokers,
                           const double* pLeadNwOut, const int32_t* topicCountDense) {
  DeviceGuard dg(ordinal_);
  stopServer();
  for (int b = 0; b < B_; ++b) {
    BrokerRec& x = hBrokers_[b];
    for (int k = 0; k < 4; ++k) x.util[k] = bUtilRM[(size_t)k * B_ + b];
    x.nrep = bNrep[b];
    x.nlead = bNlead[b];
    x.pot = bPot[b];
    x.lbi = bLeadNwIn[b];
    x.alive = bAlive[b];
    x.allowedBits = allowedHost_[b];
    for (int k = 0; k < 3; ++k) x.hutil[k] = x.util[k];  // a host of its own (uploadHosts otherwise)
  }
  std::vector<ReplicaRec> reps(R_);
  for (int r = 0; r < R_; ++r) {
    ReplicaRec& x = reps[r];
    std::memset(&x, 0, sizeof(x));
    for (int k = 0; k < 4; ++k) x.util[k] = rUtilRM[(size_t)k * R_ + r];
    x.broker = rBroker[r];
    x.part = hRPart_[r];
    x.orig = hROrig_[r];
    x.flags = rFlags[r] | (bAlive[hROrig_[r]] ? 0 : RF_ORIG_DEAD);
  }
  for (int p = 0; p < P_; ++p) {
    PartitionRec& x = hParts_[p];
    for (int k = 0; k < kMaxRf; ++k) {
      const bool in = k < x.n;
      x.brokers[k] = in ? pBrokers[hPOff_[p] + k] : -1;
      x.racks[k] = (int16_t)(in ? bRackHost_[x.brokers[k]] : -1);
    }
    x.leadNwOut = pLeadNwOut[p];
  }
  hipCheck(hipMemcpy(brokers_, hBrokers_.data(), sizeof(BrokerRec) * B_, hipMemcpyHostToDevice), "upload brokers");
  hipCheck(hipMemcpy(replicas_, reps.data(), sizeof(ReplicaRec) * R_, hipMemcpyHostToDevice), "upload replicas");
  hipCheck(hipMemcpy(parts_, hParts_.data(), sizeof(PartitionRec) * P_, hipMemcpyHostToDevice), "upload partitions");
  hipCheck(hipMemcpy(topicCount_, topicCountDense, sizeof(int32_t) * (size_t)T_ * ldB_, hipMemcpyHostToDevice),
           "upload topicCount");
  hRPart_.clear();
  hROrig_.clear();
}

void Device::uploadHosts(const double* hutil, const double* hcap) {
  DeviceGuard dg(ordinal_);
  stopServer();
  for (int b = 0; b < B_; ++b)
    for (int k = 0; k < 3; ++k) hBrokers_[b].hutil[k] = hutil[3 * (size_t)b + k];
  hipCheck(hipMemcpy(brokers_, hBrokers_.data(), sizeof(BrokerRec) * B_, hipMemcpyHostToDevice), "upload brokers");
  if (!hostCap_) hipCheck(hipMalloc((void**)&hostCap_, sizeof(double) * 3 * (size_t)B_), "hipMalloc hostCap");
  hipCheck(hipMemcpy(hostCap_, hcap, sizeof(double) * 3 * (size_t)B_, hipMemcpyHostToDevice), "upload hostCap");
}

void Device::setAllowed(int slot, const uint8_t* allowedB) {
  DeviceGuard dg(ordinal_);
  stopServer();
  if (slot < 0 || slot >= G_) throw std::runtime_error("goal slot out of range");
  for (int b = 0; b < B_; ++b)
    allowedHost_[b] = (allowedHost_[b] & ~(1u << slot)) | (allowedB[b] ? (1u << slot) : 0u);
  // strided write of BrokerRec::allowedBits (the rest of every record is left alone)
  hipCheck(hipMemcpy2DAsync(&brokers_[0].allowedBits, sizeof(BrokerRec), allowedHost_.data(), sizeof(uint32_t),
                            sizeof(uint32_t), B_, hipMemcpyHostToDevice, ST),
           "upload allowed");
  hipCheck(hipStreamSynchronize(ST), "sync");
}

void Device::setExclusions(const uint8_t* exclLead, const uint8_t* exclMove, const uint8_t* isNew) {
  DeviceGuard dg(ordinal_);
  stopServer();
  const uint32_t mask = (1u << kExclLeadBit) | (1u << kExclMoveBit) | (1u << kNewBit);
  for (int b = 0; b < B_; ++b)
    allowedHost_[b] = (allowedHost_[b] & ~mask) | (exclLead[b] ? (1u << kExclLeadBit) : 0u) |
                      (exclMove[b] ? (1u << kExclMoveBit) : 0u) | (isNew[b] ? (1u << kNewBit) : 0u);
  hipCheck(hipMemcpy2DAsync(&brokers_[0].allowedBits, sizeof(BrokerRec), allowedHost_.data(), sizeof(uint32_t),
                            sizeof(uint32_t), B_, hipMemcpyHostToDevice, ST),
           "upload exclusions");
  hipCheck(hipStreamSynchronize(ST), "sync");
}

void Device::setTopicLimits(const int32_t* upper, const int32_t* lower) {
  DeviceGuard dg(ordinal_);
  stopServer();
  hipCheck(hipMemcpyAsync(tUpper_, upper, sizeof(int32_t) * T_, hipMemcpyHostToDevice, ST), "upload tUpper");
  hipCheck(hipMemcpyAsync(tLower_, lower, sizeof(int32_t) * T_, hipMemcpyHostToDevice, ST), "upload tLower");
  hipCheck(hipStreamSynchronize(ST), "sync");
}

void Device::enableTopicLeaders(const int32_t* dense) {
  DeviceGuard dg(ordinal_);
  stopServer();
  if (!topicLead_) dalloc(&topicLead_, (size_t)T_ * ldB_);
  hipCheck(hipMemcpy(topicLead_, dense, sizeof(int32_t) * (size_t)T_ * ldB_, hipMemcpyHostToDevice), "upload topicLead");
}

void Device::setMinLeaders(const int32_t* tMin) {
  DeviceGuard dg(ordinal_);
  stopServer();
  if (!tMinLead_) dalloc(&tMinLead_, (size_t)T_);
  hipCheck(hipMemcpy(tMinLead_, tMin, sizeof(int32_t) * (size_t)T_, hipMemcpyHostToDevice), "upload tMinLead");
}

void Device::setTopicLeadLimits(const int32_t* lim) {
  DeviceGuard dg(ordinal_);
  stopServer();
  if (!tLeadLim_) dalloc(&tLeadLim_, 2 * (size_t)T_);
  hipCheck(hipMemcpy(tLeadLim_, lim, sizeof(int32_t) * 2 * (size_t)T_, hipMemcpyHostToDevice), "upload tLeadLim");
}

void Device::setBrokerSets(const int32_t* brokerSet, const int32_t* replicaSet) {
  DeviceGuard dg(ordinal_);
  stopServer();
  hipCheck(hipMemcpy2DAsync(&brokers_[0].bset, sizeof(BrokerRec), brokerSet, sizeof(int32_t), sizeof(int32_t), B_,
                            hipMemcpyHostToDevice, ST),
           "upload broker sets");
  hipCheck(hipMemcpy2DAsync(&replicas_[0].bset, sizeof(ReplicaRec), replicaSet, sizeof(int32_t), sizeof(int32_t), R_,
                            hipMemcpyHostToDevice, ST),
           "upload replica broker sets");
  hipCheck(hipStreamSynchronize(ST), "sync");
}

size_t Device::updatesBytes() const {
  return align16(brows.size() * sizeof(BrokerRow)) + align16(rrows.size() * sizeof(ReplicaRow)) +
         align16(prows.size() * sizeof(PartitionRow)) + align16(tdeltas.size() * sizeof(TopicCountDelta));
}

// [broker rows | replica rows | partition rows | topic deltas] at the start of the staging area
Device::Staged Device::packUpdates(size_t extra) {
  Staged g;
  g.nb = (int)brows.size();
  g.nr = (int)rrows.size();
  g.np = (int)prows.size();
  g.nt = (int)tdeltas.size();
  stageUsed_ = 0;
  ensureStage(updatesBytes() + extra + 64);
  g.obr = 0;
  std::memcpy(hStage_ + g.obr, brows.data(), g.nb * sizeof(BrokerRow));
  g.orr = g.obr + align16(g.nb * sizeof(BrokerRow));
  std::memcpy(hStage_ + g.orr, rrows.data(), g.nr * sizeof(ReplicaRow));
  g.opr = g.orr + align16(g.nr * sizeof(ReplicaRow));
  std::memcpy(hStage_ + g.opr, prows.data(), g.np * sizeof(PartitionRow));
  g.otd = g.opr + align16(g.np * sizeof(PartitionRow));
  std::memcpy(hStage_ + g.otd, tdeltas.data(), g.nt * sizeof(TopicCountDelta));
  g.end = g.otd + align16(g.nt * sizeof(TopicCountDelta));
  brows.clear();
  rrows.clear();
  prows.clear();
  tdeltas.clear();
  stageUsed_ = g.end;
  return g;
}

// Put staged rows back into the pending lists (a scan the server declined goes through packUpdates again).
void Device::unpackUpdates(const Staged& g) {
  brows.assign((const BrokerRow*)(hStage_ + g.obr), (const BrokerRow*)(hStage_ + g.obr) + g.nb);
  rrows.assign((const ReplicaRow*)(hStage_ + g.orr), (const ReplicaRow*)(hStage_ + g.orr) + g.nr);
  prows.assign((const PartitionRow*)(hStage_ + g.opr), (const PartitionRow*)(hStage_ + g.opr) + g.np);
  tdeltas.assign((const TopicCountDelta*)(hStage_ + g.otd), (const TopicCountDelta*)(hStage_ + g.otd) + g.nt);
}

// One `prep` launch: apply the staged rows, copy `reqBytes` of request (staged at g.end) into HBM, and (for a
// scan) reset the result words and the arrival counter.
void Device::launchPrepFor(const Staged& g, size_t reqBytes, bool scan) {
  stopServer();
  const int nReq4 = (int)(align16(reqBytes) / 16);
  if (nReq4) ensureReq((size_t)nReq4 * 16);
  hipCheck(launchPrep(mutTables(), stagedList(g), (const int4*)(hStageDev_ + g.end), (int4*)dReq_, nReq4,
                      scan ? dResult_ : nullptr, scan ? dDone_ : nullptr, ST),
           "prep");
}

// Spin on the host-mapped mailbox for `seq`; a stream error (or a stream that drained without publishing)
// is reported instead of spinning forever. With `serverCmd`, a server that its idle watchdog ended before it saw the
// command (exit record {1, seq - 1}) returns false instead.
bool Device::waitMail(unsigned long long seq, bool serverCmd) {
  PhaseScope ps(PH_SCAN_WAIT);
  volatile unsigned long long* mail = hResult_;
  const unsigned long long want = seq & 0xffffffffull;
  uint64_t spins = 0;
  bool idle = (bool)idleWork;
  while ((__atomic_load_n(&mail[0], __ATOMIC_ACQUIRE) >> 32) != want) {
    if (idle) {  // the engine's speculative host work, one unit per poll
      idle = idleWork();
      continue;
    }
    // the stream is asked whether the kernel ended without publishing (a server's watchdog exit, a park, a fault) only
    // after ~16 K polls (~0.2 ms, ten round trips) and then every 1 K: a runtime call in the middle of an ordinary wait
    // would hold up noticing the result that lands meanwhile
    if ((++spins & 1023) == 0 && spins >= spinsBeforeQuery_) {
      const hipError_t q = hipStreamQuery(ST);
      if (q == hipSuccess) {
        if ((__atomic_load_n(&mail[0], __ATOMIC_ACQUIRE) >> 32) == want) break;
        const unsigned long long ex = __atomic_load_n(&mail[3], __ATOMIC_ACQUIRE);
        if (serverCmd && (ex >> 32) == 1 && (ex & 0xffffffffull) == ((seq - 1) & 0xffffffffull)) return false;
        if (serverCmd && (ex >> 32) == 5 && (ex & 0xffffffffull) == want) {
          // the server parked with this command waiting for a shard group: its result still arrives in mail[0]
          parkedPending_ = true;
          const double t0 = nowSeconds();
          for (uint64_t k = 0; (__atomic_load_n(&mail[0], __ATOMIC_ACQUIRE) >> 32) != want; ++k) {
            if ((k & 4095) == 4095 && nowSeconds() - t0 > 120.0)
              throw std::runtime_error("shard group combine: not every rank arrived (120 s)");
            if (k > (1u << 16)) sched_yield();
            else __builtin_ia32_pause();
          }
          break;
        }
        char msg[256];
        std::snprintf(msg, sizeof(msg),
                      "scan finished without publishing its result (seq %llu, mail %016llx, server %s, server exit "
                      "%016llx)",
                      (unsigned long long)seq, (unsigned long long)mail[0], serverOn_ ? "on" : "off",
                      (unsigned long long)mail[3]);
        throw std::runtime_error(msg);
      }
      if (q != hipErrorNotReady) hipCheck(q, "scan");
    }
    // a scan is ~10-30 us; past ~1 ms of spinning the host core is yielded between polls so concurrent sessions
    // (and the JVM's own threads) get it back
    if (spins > (1u << 16)) sched_yield();
    else __builtin_ia32_pause();
  }
  perf.syncs++;
  return true;
}

// A shard with nothing to scan still applies its pending row updates so every shard's tables stay identical.
void Device::flushPending() {
  DeviceGuard dg(ordinal_);
  if (!brows.empty() || !rrows.empty() || !prows.empty() || !tdeltas.empty()) flushOnly();
}

void Device::flushOnly() {
  DeviceGuard dg(ordinal_);
  stopServer();
  if (brows.empty() && rrows.empty() && prows.empty() && tdeltas.empty()) return;
  const Staged g = packUpdates(0);
  launchPrepFor(g, 0, false);
  hipCheck(hipStreamSynchronize(ST), "sync");
  perf.syncs++;
}

int64_t Device::finishScan() {
  waitMail(seq_);
  if (timing) {
    hipCheck(hipEventSynchronize(EV1), "hipEventSynchronize");
    float ms = 0.f;
    hipCheck(hipEventElapsedTime(&ms, EV0, EV1), "hipEventElapsedTime");
    perf.scanKernelMs += ms;
  }
  const unsigned long long lo = hResult_[0] & 0xffffffffull;  // key + 1, 0 = no winner
  return lo == 0 ? -1 : (int64_t)(lo - 1);
}

// A cross/pair scan is one launch when its update list fits the kernel's LDS overlay and its request is
// small enough to read straight from host memory; otherwise `prep` applies the rows and copies the request
// into HBM first.
// Requests are read by the scan straight from the host-mapped staging area (rows that lose to an earlier winner
// are never read, so copying the request into HBM first would only add a launch and a full PCIe read).
constexpr size_t kDirectRequestBytes = 8 << 20;

UpdateList Device::stagedList(const Staged& g) const { return overlayFor(g); }

UpdateList Device::overlayFor(const Staged& g) const {
  UpdateList u;
  u.brows = (const BrokerRow*)(hStageDev_ + g.obr);
  u.rrows = (const ReplicaRow*)(hStageDev_ + g.orr);
  u.prows = (const PartitionRow*)(hStageDev_ + g.opr);
  u.tdel = (const TopicCountDelta*)(hStageDev_ + g.otd);
  u.nb = g.nb;
  u.nr = g.nr;
  u.np = g.np;
  u.nt = g.nt;
  return u;
}

MutTables Device::mutTables() const {
  return MutTables{brokers_, replicas_, parts_, topicCount_, topicLead_, ldB_};
}

// Returns the request base the scan reads (host-mapped staging or the HBM copy) and the update list it
// applies itself (empty when prep ran).
// Topic-count deltas are atomics applied by workgroup 0 during the launch, so a program that reads topic counts
// always has them applied by `prep` first.
const char* Device::stageScan(const Staged& g, size_t req, bool readsTopicCounts, UpdateList& u) {
  const bool fits = g.nb <= kOverlayRows && g.nr <= kOverlayRows && g.np <= kOverlayRows &&
                    !(readsTopicCounts && g.nt > 0);
  if (fits && req <= kDirectRequestBytes) {
    u = overlayFor(g);
    perf.singleLaunch++;
    return hStageDev_ + g.end;
  }
  launchPrepFor(g, req, false);
  u = UpdateList{nullptr, nullptr, nullptr, nullptr, 0, 0, 0, 0};
  return dReq_;
}

int64_t Device::scanCross(const DevProgram& prog, const int32_t* reps, int K, const int32_t* cands, int N, int c0,
                          int c1) {
  DeviceGuard dg(ordinal_);
  const int Nr = c1 - c0;
  if (K <= 0 || Nr <= 0) {
    flushPending();
    return -1;
  }
  if ((uint64_t)K * (uint64_t)N >= (1ull << 31)) throw std::runtime_error("scan too large");
  const size_t oCand = (size_t)K * sizeof(RowRef);
  const size_t req = oCand + align16((size_t)Nr * 4);
  const bool readsTc = (prog.needs & (NEED_TOPIC | NEED_TLEAD)) != 0;
  {
    bool serve = false;
    const Staged g = packForServer(prog, readsTc, serve);
    if (serve) {
      const int32_t params[6] = {K, Nr, N, c0, Nr >= (int)scanXcdSliceMinCols() ? 1 : 0, 0};
      const int64_t key = serverRun(prog, g, SOP_CROSS, reps, (size_t)K, cands + c0, (size_t)Nr, params);
      if (key != INT64_MIN) {
        perf.scanPairs += (int64_t)K * Nr;
        perf.scanBytes += (int64_t)K * Nr * kBytesPerCandidate;
        const int64_t required = key < 0 ? (int64_t)K * Nr : (key / N) * Nr + (key % N - c0) + 1;
        perf.scanRequired += required;
        perf.serverRequired += required;
        perf.crossRequired += required;
        prof().count(24, "req.cross", required);
        return key;
      }
    }
    unpackUpdates(g);
  }
  stopServer();
  UpdateList u;
  const char* base;
  {
    PhaseScope ps(PH_SCAN_STAGE);
    const Staged g = packUpdates(req);
    writeRowRefs(hStage_ + g.end, reps, (size_t)K);
    std::memcpy(hStage_ + g.end + oCand, cands + c0, (size_t)Nr * 4);
    base = stageScan(g, req, readsTc, u);
  }
  ++seq_;
  if (timing) (void)hipEventRecord(EV0, ST);
  hipCheck(launchScanCross(tables(), mutTables(), u, prog, (const RowRef*)base, (const int32_t*)(base + oCand), K, Nr,
                           N, c0, dResult_, dDone_, hResultDev_, seq_, ST),
           "scan_cross");
  if (timing) (void)hipEventRecord(EV1, ST);
  perf.scanLaunches++;
  perf.scanPairs += (int64_t)K * Nr;
  perf.scanBytes += (int64_t)K * Nr * kBytesPerCandidate;
  const double ms0 = perf.scanKernelMs;
  const int64_t key = finishScan();
  // candidates this launch had to evaluate: every row before the winner's and the winner's row up to the winner
  const int64_t required = key < 0 ? (int64_t)K * Nr : (key / N) * Nr + (key % N - c0) + 1;
  perf.scanRequired += required;
  perf.crossLaunches++;
  perf.crossRequired += required;
  perf.crossKernelMs += perf.scanKernelMs - ms0;
  return key;
}

int64_t Device::scanSwap(const DevProgram& prog, const int32_t* srcs, int S, const int32_t* cbOff, int M,
                         const int32_t* cbRep, int nCand, const SwapLimit& lim, int64_t* visited) {
  DeviceGuard dg(ordinal_);
  stopServer();
  *visited = 0;
  if (S <= 0 || M <= 0 || nCand <= 0) return -1;
  const size_t rows = (size_t)S * M;
  if (rows > rowVisitedCap_) {
    if (rowVisited_) (void)hipFree(rowVisited_);
    rowVisitedCap_ = rows * 2;
    hipCheck(hipMalloc((void**)&rowVisited_, rowVisitedCap_ * sizeof(int32_t)), "hipMalloc rowVisited");
  }
  const size_t oOff = align16((size_t)S * 4);
  const size_t oRep = oOff + align16((size_t)(M + 1) * 4);
  const size_t req = oRep + align16((size_t)nCand * 4);
  const Staged g = packUpdates(req);
  std::memcpy(hStage_ + g.end, srcs, (size_t)S * 4);
  std::memcpy(hStage_ + g.end + oOff, cbOff, (size_t)(M + 1) * 4);
  std::memcpy(hStage_ + g.end + oRep, cbRep, (size_t)nCand * 4);
  launchPrepFor(g, req, true);
  ++seq_;
  hipCheck(launchScanSwap(tables(), prog, (const int32_t*)dReq_, S, (const int32_t*)(dReq_ + oOff),
                          (const int32_t*)(dReq_ + oRep), M, lim, dResult_, rowVisited_, hResultDev_, seq_, ST,
                          timing ? EV0 : nullptr, timing ? EV1 : nullptr),
           "scan_swap");
  perf.scanLaunches++;
  perf.scanPairs += (int64_t)S * nCand;
  perf.scanBytes += (int64_t)S * nCand * kBytesPerCandidate;
  (void)finishScan();
  const unsigned long long best = hResult_[1];
  *visited = (int64_t)hResult_[2];
  perf.scanRequired += *visited;
  return best == ~0ull ? -1 : (int64_t)best;
}

int64_t Device::scanPairs(const DevProgram& prog, const int32_t* pr, const int32_t* pb, int p0, int p1) {
  DeviceGuard dg(ordinal_);
  const int n = p1 - p0;
  if (n <= 0) {
    flushPending();
    return -1;
  }
  const size_t oB = (size_t)n * sizeof(RowRef);
  const size_t req = oB + align16((size_t)n * 4);
  const bool readsTc = (prog.needs & (NEED_TOPIC | NEED_TLEAD)) != 0;
  {
    bool serve = false;
    const Staged g0 = packForServer(prog, readsTc, serve);
    if (serve) {
      const int32_t params[6] = {n, p0, 0, 0, 0, 0};
      const int64_t key = serverRun(prog, g0, SOP_PAIRS, pr + p0, (size_t)n, pb + p0, (size_t)n, params);
      if (key != INT64_MIN) {
        perf.scanPairs += n;
        perf.scanBytes += (int64_t)n * kBytesPerCandidate;
        const int64_t required = key < 0 ? (int64_t)n : key - p0 + 1;
        perf.scanRequired += required;
        perf.serverRequired += required;
        prof().count(25, "req.pairs", required);
        return key;
      }
    }
    unpackUpdates(g0);
  }
  stopServer();
  const Staged g = packUpdates(req);
  writeRowRefs(hStage_ + g.end, pr + p0, (size_t)n);
  std::memcpy(hStage_ + g.end + oB, pb + p0, (size_t)n * 4);
  UpdateList u;
  const char* base = stageScan(g, req, readsTc, u);
  ++seq_;
  if (timing) (void)hipEventRecord(EV0, ST);
  hipCheck(launchScanPairs(tables(), mutTables(), u, prog, (const RowRef*)base, (const int32_t*)(base + oB), n, p0,
                           dResult_, dDone_, hResultDev_, seq_, ST),
           "scan_pairs");
  if (timing) (void)hipEventRecord(EV1, ST);
  perf.scanLaunches++;
  perf.scanPairs += n;
  perf.scanBytes += (int64_t)n * kBytesPerCandidate;
  const int64_t key = finishScan();
  perf.scanRequired += key < 0 ? (int64_t)n : key - p0 + 1;
  return key;
}

CombineBlock* Device::allocCombineBlock() {
  CombineBlock* b = nullptr;
  hipCheck(hipHostMalloc((void**)&b, sizeof(CombineBlock),
                         hipHostMallocPortable | hipHostMallocMapped | hipHostMallocCoherent),
           "hipHostMalloc shard group");
  initCombineBlock(b);
  return b;
}
void Device::freeCombineBlock(CombineBlock* b) {
  if (b) (void)hipHostFree(b);
}
void Device::attachGroup(CombineBlock* blk, int count, int rank) {
  DeviceGuard dg(ordinal_);
  void* d = nullptr;
  hipCheck(hipHostGetDevicePointer(&d, blk, 0), "hipHostGetDevicePointer shard group");
  // every rank (its server or its host thread) may publish into this rank's mailbox: one address for all of them
  if (d != (void*)blk || hResultDev_ != (unsigned long long*)hResult_)
    throw std::runtime_error("shard groups need pinned host memory at one address on host and devices");
  grpHost_ = blk;
  grpDev_ = (unsigned long long)(uintptr_t)d;
  grpCount_ = count;
  grpRank_ = rank;
  grpCalls_ = 0;
  grpHostSeq_ = 0;
  devCombined_ = false;
  __atomic_store_n(&hResult_[6], 0ull, __ATOMIC_RELAXED);
  __atomic_store_n(&blk->mail[rank], (unsigned long long)(uintptr_t)hResult_, __ATOMIC_RELEASE);
}
int64_t Device::groupCombineHost(int64_t key) {
  const int slot = (int)(grpCalls_ & 1);
  ++grpCalls_;
  return groupHostMin(grpHost_, slot, grpRank_, grpCount_, key, ++grpHostSeq_, 120.0);
}

int64_t Device::segUpload(const SegIn& sg) {
  const void* key = sg.v.get();
  auto it = segCache_.find(key);
  if (it != segCache_.end()) return it->second.second;
  const size_t n = sg.v->size();
  const size_t span = (n + 7) & ~(size_t)7;  // whole 128-byte lines: no line holds rows of two uploads
  if (span > segCap_) return -1;
  if (segHead_ + span > segCap_) {
    // wrap: the server is restarted before any reused line is read (a launch starts with clean caches)
    stopServer();
    segCache_.clear();
    segHead_ = 0;
    ++poolEpoch_;  // every queue-directory entry now points at rows that will be overwritten
  }
  if (n) {
    for (int r : *sg.v)
      if (rowBroker_[r] != sg.cb) throw std::logic_error("snapshot segment is not current for its broker");
    writeRowRefs((char*)(segPool_ + segHead_), sg.v->data(), n);
    perf.serverPayloadBytes += (int64_t)(n * sizeof(RowRef));
    prof().addPayload((int64_t)(n * sizeof(RowRef)));
    prof().count(14, "srv.bytes.pool", (int64_t)(n * sizeof(RowRef)));
  }
  const uint32_t off = (uint32_t)segHead_;
  segHead_ += span;
  segCache_.emplace(key, std::make_pair(sg.v, off));
  return off;
}

bool Device::queueUsable() const { return serverUsable_ && serverAllowed_; }

void Device::qdirBind(uint64_t key) {
  if (key == qdirKey_ && qdir_) return;
  qdirKey_ = key;
  qdirSpan_ = 1;
  qdirSnap_.assign(B_, nullptr);
  if (!qdir_) {
    DeviceGuard dg(ordinal_);
    hipCheck(hipExtMallocWithFlags((void**)&qdir_, sizeof(QueueDirEntry) * (size_t)B_, hipDeviceMallocFinegrained),
             "hipExtMallocWithFlags queue directory");
  }
}

bool Device::qdirSet(int b, std::shared_ptr<const std::vector<int32_t>> v) {
  if (!qdir_ || b < 0 || b >= B_) throw std::logic_error("qdirSet before qdirBind");
  if (v->size() >= (1u << 20)) return false;
  const int64_t off = segUpload(SegIn{v, b, 0});
  if (off < 0) return false;
  // a plain 8-byte store through the BAR; the command that reads it is published behind a store fence
  QueueDirEntry e{(uint32_t)off, (int32_t)v->size()};
  *reinterpret_cast<volatile unsigned long long*>(&qdir_[b]) = *reinterpret_cast<const unsigned long long*>(&e);
  qdirSpan_ = std::max(qdirSpan_, (int)v->size());
  qdirSnap_[b] = std::move(v);
  return true;
}

bool Device::qdirSetMany(const std::vector<int32_t>& bs,
                         const std::vector<std::shared_ptr<const std::vector<int32_t>>>& snaps) {
  const int n = (int)bs.size();
  if (!qdir_ || (int)snaps.size() != n) throw std::logic_error("qdirSetMany before qdirBind");
  if (n < 8) {
    for (int i = 0; i < n; ++i)
      if (!qdirSet(bs[i], snaps[i])) return false;
    return true;
  }
  auto spanOf = [](size_t k) { return (k + 7) & ~(size_t)7; };  // whole 128-byte lines, as segUpload
  std::vector<int64_t> off(n, -1);
  std::vector<uint8_t> fresh(n, 0);
  auto assign = [&]() {
    size_t need = 0;
    for (int i = 0; i < n; ++i) {
      const auto it = segCache_.find(snaps[i].get());
      fresh[i] = it == segCache_.end();
      off[i] = fresh[i] ? -1 : (int64_t)it->second.second;
      if (fresh[i]) need += spanOf(snaps[i]->size());
    }
    return need;
  };
  for (const auto& v : snaps)
    if (v->size() >= (1u << 20)) return false;
  size_t need = assign();
  if (need > segCap_) return false;
  if (segHead_ + need > segCap_) {  // wrap first (as segUpload): the listed entries are rewritten from the pool start
    stopServer();
    segCache_.clear();
    segHead_ = 0;
    ++poolEpoch_;
    // every snapshot is fresh after the wrap: the whole directory may not fit even though its uncached part did
    need = assign();
    if (need > segCap_) return false;
  }
  for (int i = 0; i < n; ++i)
    if (fresh[i]) {
      off[i] = (int64_t)segHead_;
      segHead_ += spanOf(snaps[i]->size());
    }
  std::atomic<int> stale{-1};
  HostPool::get().parallelFor(n, [&](int i) {
    if (!fresh[i] || snaps[i]->empty()) return;
    for (int r : *snaps[i])
      if (rowBroker_[r] != bs[i]) stale.store(bs[i]);
    writeRowRefs((char*)(segPool_ + off[i]), snaps[i]->data(), snaps[i]->size());
  });
  if (stale.load() >= 0) throw std::logic_error("snapshot segment is not current for its broker");
  for (int i = 0; i < n; ++i) {
    const int b = bs[i];
    const auto& v = snaps[i];
    if (fresh[i]) {
      segCache_.emplace(v.get(), std::make_pair(v, (uint32_t)off[i]));
      perf.serverPayloadBytes += (int64_t)(v->size() * sizeof(RowRef));
      prof().addPayload((int64_t)(v->size() * sizeof(RowRef)));
      prof().count(14, "srv.bytes.pool", (int64_t)(v->size() * sizeof(RowRef)));
    }
    QueueDirEntry e{(uint32_t)off[i], (int32_t)v->size()};
    *reinterpret_cast<volatile unsigned long long*>(&qdir_[b]) = *reinterpret_cast<const unsigned long long*>(&e);
    qdirSpan_ = std::max(qdirSpan_, (int)v->size());
    qdirSnap_[b] = v;
  }
  return true;
}

int64_t Device::scanQueue(const DevProgram& prog, int head, int skip0, const int32_t* tail, int nTail,
                          const int32_t* cands, int N) {
  DeviceGuard dg(ordinal_);
  const int hasHead = head >= 0 ? 1 : 0;
  const int n = hasHead + nTail;
  if (n <= 0 || N <= 0) return -1;
  auto entry = [&](int i) { return i < hasHead ? head : tail[i - hasHead]; };
  const int span = qdirSpan_;
  const uint64_t space = (uint64_t)n * (uint64_t)span * (uint64_t)N;
  if (queueUsable() && space < (1ull << 31)) {
    bool serve = false;
    const bool readsTc = (prog.needs & (NEED_TOPIC | NEED_TLEAD)) != 0;
    const Staged g = packForServer(prog, readsTc, serve);
    if (serve) {
      const size_t oRows = align16(sizeof(DevProgram));
      const size_t oA = oRows + g.end, oC = oA + align16((size_t)n * 4), end = oC + align16((size_t)N * 4);
      ensureFg(kCmdBytes + end);
      if (ensureServer()) {
        char* pay = fg_ + kCmdBytes;
        const int ver = serverProgram(prog, pay);
        if (g.end) std::memcpy(pay + oRows, hStage_, g.end);
        if (hasHead) std::memcpy(pay + oA, &head, 4);
        std::memcpy(pay + oA + 4 * (size_t)hasHead, tail, (size_t)nTail * 4);
        std::memcpy(pay + oC, cands, (size_t)N * 4);
        perf.serverPayloadBytes += (int64_t)(g.end + (size_t)n * 4 + (size_t)N * 4);
        prof().addPayload((int64_t)(g.end + (size_t)n * 4 + (size_t)N * 4));
        prof().count(12, "srv.bytes.A", (int64_t)n * 4);
        ServerCmd c;
        std::memset(&c, 0, sizeof(c));
        c.op = SOP_QUEUE;
        c.n = n;
        c.K = span;
        c.N = N;
        c.c0 = skip0;
        c.progVer = ver;
        // one wave per candidate (a tile of kBlock slots): the queue is usually hundreds of brokers deep, so the scan
        // is a few sweeps of every workgroup and the sweeps, not a single tile's conjunction, are its latency
        c.goalParts = 1;
        // (no adaptive width here: queue winners' depths vary too much from one command to the next — sized from the
        // deepest of the last 8 winners, the extra sweeps cost 26 us per queue command on C2 against 0.25 GB less
        // traffic, profiles/r05/README.md)
        c.nActive = std::min(serverBlocks_, std::max(8, (n + 7) / 8 * 8));
        c.nb = g.nb;
        c.nr = g.nr;
        c.np = g.np;
        c.nt = g.nt;
        c.oProg = 0;
        c.oB = (uint32_t)(oRows + g.obr);
        c.oR = (uint32_t)(oRows + g.orr);
        c.oP = (uint32_t)(oRows + g.opr);
        c.oT = (uint32_t)(oRows + g.otd);
        c.oA = (uint32_t)oA;
        c.oC = (uint32_t)oC;
        c.queueDir = (unsigned long long)(uintptr_t)qdir_;
        const auto tq = std::chrono::steady_clock::now();
        if (postCommand(c, (g.nb | g.nr | g.np | g.nt) != 0)) {
          perf.serverScans++;
          const unsigned long long lo = hResult_[0] & 0xffffffffull;
          const int64_t key = lo == 0 ? -1 : (int64_t)(lo - 1);
          if (prof().on) {  // CCMI_PROFILE: queue commands' round trips and depths
            prof().count(21, "queue.wait.ns",
                         (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - tq)
                             .count());
            prof().count(22, "queue.scans", 1);
            prof().count(23, "queue.entries.before.winner", key < 0 ? n : key / N / span);
          }
          // required candidates: every row before the winner's, then the winner's columns up to it (device-side
          // accounting only: the scan's evaluated pair space is not walked here)
          int64_t required = 0, K = 0;
          const int wi = key < 0 ? n : (int)(key / N / span);
          for (int i = 0; i < wi; ++i) {
            const int len = qdirLen(entry(i)), s0 = i == 0 ? skip0 : 0;
            required += len > s0 ? (int64_t)(len - s0) * N : 0;
          }
          if (key >= 0) required += ((key / N) % span - (wi == 0 ? skip0 : 0)) * N + key % N + 1;
          K = required;  // pairs the device had to evaluate (speculative tiles past the winner not counted)
          perf.scanPairs += K;
          perf.scanBytes += K * kBytesPerCandidate;
          perf.scanRequired += required;
          perf.serverRequired += required;
          perf.crossRequired += required;
          prof().count(27, "req.queue", required);
          return key;
        }
      }
    }
    unpackUpdates(g);
  }
  // no server (or too many keys): the rows flattened for a plain cross scan, its key mapped back
  segFlat_.clear();
  std::vector<int32_t> entryOf, rowOf;
  for (int i = 0; i < n; ++i) {
    const auto& v = *qdirSnap_[entry(i)];
    for (size_t r = i == 0 ? (size_t)skip0 : 0; r < v.size(); ++r) {
      segFlat_.push_back(v[r]);
      entryOf.push_back(i);
      rowOf.push_back((int32_t)r);
    }
  }
  if (segFlat_.empty()) return -1;
  const int64_t k = scanCross(prog, segFlat_.data(), (int)segFlat_.size(), cands, N, 0, N);
  if (k < 0) return -1;
  const int64_t fr = k / N;
  return ((int64_t)entryOf[fr] * span + rowOf[fr]) * N + k % N;
}

int64_t Device::scanSegs(const DevProgram& prog, const std::vector<SegIn>& segs, const int32_t* cands, int N, int c0,
                         int c1) {
  DeviceGuard dg(ordinal_);
  const int Nr = c1 - c0;
  size_t K = 0;
  for (const SegIn& sg : segs) K += sg.v->size() > sg.skip ? sg.v->size() - sg.skip : 0;
  const bool readsTc = (prog.needs & (NEED_TOPIC | NEED_TLEAD)) != 0;
  bool served = serverUsable_ && serverAllowed_ && K > 0 && Nr > 0 && segs.size() <= (size_t)kMaxSegs &&
                (uint64_t)K * (uint64_t)N < (1ull << 31);
  // A pool wrap while uploading segment j rewrites the pool from its start, so the offsets of segments 0..j-1 may
  // name overwritten rows: the table is rebuilt once from the emptied pool, and a second wrap means the segments do
  // not fit the pool together (the flat path below).
  for (int attempt = 0; served && attempt < 2; ++attempt) {
    const auto epoch = poolEpoch_;
    segTab_.clear();
    int32_t start = 0;
    for (const SegIn& sg : segs) {
      const int64_t off = segUpload(sg);
      if (off < 0) {
        served = false;
        break;
      }
      const size_t len = sg.v->size() > sg.skip ? sg.v->size() - sg.skip : 0;
      segTab_.push_back(SegEntry{(uint32_t)(off + (int64_t)std::min(sg.skip, sg.v->size())), start});
      start += (int32_t)len;
    }
    segTab_.push_back(SegEntry{0, start});
    if (!served || poolEpoch_ == epoch) break;
    if (attempt == 1) served = false;
  }
  if (served) {
    bool serve = false;
    const Staged g = packForServer(prog, readsTc, serve);
    if (serve) {
      const int S = (int)segs.size();
      const int32_t params[6] = {(int32_t)K, Nr, N, c0, Nr >= (int)scanXcdSliceMinCols() ? 1 : 0, S};
      const int64_t key = serverRun(prog, g, SOP_SEGS, segTab_.data(), (size_t)S + 1, cands + c0, (size_t)Nr, params);
      if (key != INT64_MIN) {
        perf.scanPairs += (int64_t)K * Nr;
        perf.scanBytes += (int64_t)K * Nr * kBytesPerCandidate;
        const int64_t required = key < 0 ? (int64_t)K * Nr : (key / N) * Nr + (key % N - c0) + 1;
        perf.scanRequired += required;
        perf.serverRequired += required;
        perf.crossRequired += required;
        prof().count(26, "req.segs", required);
        return key;
      }
    }
    unpackUpdates(g);
  }
  segFlat_.clear();
  for (const SegIn& sg : segs)
    if (sg.v->size() > sg.skip) segFlat_.insert(segFlat_.end(), sg.v->begin() + sg.skip, sg.v->end());
  return scanCross(prog, segFlat_.data(), (int)segFlat_.size(), cands, N, c0, c1);
}

void Device::stats(const StatsParams& P, const uint8_t* allowedAliveHost, StatsOut* out) {
  DeviceGuard dg(ordinal_);
  stopServer();
  const size_t req = align16((size_t)ldB_);
  const Staged g = packUpdates(req);
  std::memcpy(hStage_ + g.end, allowedAliveHost, (size_t)ldB_);
  launchPrepFor(g, req, false);
  hipCheck(hipMemcpyAsync(allowedAlive_, dReq_, (size_t)ldB_, hipMemcpyDeviceToDevice, ST), "allowedAlive");
  StatsParams Ph = P;
  Ph.hostCap = hostCap_;
  hipCheck(launchStats(Ph, topicCount_, topicNrep_, brokers_, allowedAlive_, (TopicPartial*)topicScratch_,
                       statsPart_, (StatsOut*)statsOut_, ldB_, ST, timing ? EV0 : nullptr, timing ? EV1 : nullptr),
           "stats");
  hipCheck(hipMemcpyAsync(statsHost_, statsOut_, sizeof(StatsOut), hipMemcpyDeviceToHost, ST), "D2H stats");
  hipCheck(hipStreamSynchronize(ST), "sync");
  perf.syncs++;
  perf.statsLaunches++;
  perf.statsBytes += (int64_t)T_ * ldB_ * 4 + (int64_t)ldB_ + (int64_t)T_ * 4;
  if (timing) {
    float ms = 0.f;
    hipCheck(hipEventElapsedTime(&ms, EV0, EV1), "hipEventElapsedTime");
    perf.statsKernelMs += ms;
  }
  std::memcpy((void*)out, statsHost_, sizeof(StatsOut));
}

}  // namespace ccmi

namespace ccmi {

// ------------------------------------------------------------------------------------------------ chains
void Device::uploadLoads(int W, const LoadVec* rLoad, const LoadVec* bLoad, const LoadVec* bLnw, const LoadVec* bPot,
                         const int32_t* pSlots, const int32_t* pLeader) {
  DeviceGuard dg(ordinal_);
  stopServer();
  W_ = W;
  dalloc(&dRLoad_, (size_t)R_);
  dalloc(&dBLoad_, (size_t)B_);
  dalloc(&dBLnw_, (size_t)B_);
  dalloc(&dBPot_, (size_t)B_);
  dalloc(&dPOff_, (size_t)P_ + 1);
  dalloc(&dPSlots_, (size_t)R_);
  dalloc(&dPLeader_, (size_t)P_);
  if (!hChainOut_) {
    hipCheck(hipHostMalloc((void**)&hChainOut_, sizeof(ChainResultDev), hipHostMallocMapped | hipHostMallocCoherent),
             "hipHostMalloc chain result");
    hipCheck(hipHostGetDevicePointer((void**)&hChainOutDev_, hChainOut_, 0), "hipHostGetDevicePointer");
  }
  hipCheck(hipMemcpy(dRLoad_, rLoad, sizeof(LoadVec) * R_, hipMemcpyHostToDevice), "upload replica loads");
  hipCheck(hipMemcpy(dBLoad_, bLoad, sizeof(LoadVec) * B_, hipMemcpyHostToDevice), "upload broker loads");
  hipCheck(hipMemcpy(dBLnw_, bLnw, sizeof(LoadVec) * B_, hipMemcpyHostToDevice), "upload leadership loads");
  hipCheck(hipMemcpy(dBPot_, bPot, sizeof(LoadVec) * B_, hipMemcpyHostToDevice), "upload potential loads");
  hipCheck(hipMemcpy(dPOff_, hPOff_.data(), sizeof(int32_t) * (P_ + 1), hipMemcpyHostToDevice), "upload pOff");
  hipCheck(hipMemcpy(dPSlots_, pSlots, sizeof(int32_t) * R_, hipMemcpyHostToDevice), "upload pSlots");
  hipCheck(hipMemcpy(dPLeader_, pLeader, sizeof(int32_t) * P_, hipMemcpyHostToDevice), "upload pLeader");
}

void Device::uploadHostLoads(int H, const LoadVec* hLoad, const int32_t* bHost, const int32_t* hOff,
                             const int32_t* hBrk) {
  DeviceGuard dg(ordinal_);
  stopServer();
  dalloc(&dHLoad_, (size_t)H);
  dalloc(&dBHost_, (size_t)B_);
  dalloc(&dHOff_, (size_t)H + 1);
  dalloc(&dHBrk_, (size_t)B_);
  hipCheck(hipMemcpy(dHLoad_, hLoad, sizeof(LoadVec) * H, hipMemcpyHostToDevice), "upload host loads");
  hipCheck(hipMemcpy(dBHost_, bHost, sizeof(int32_t) * B_, hipMemcpyHostToDevice), "upload broker hosts");
  hipCheck(hipMemcpy(dHOff_, hOff, sizeof(int32_t) * (H + 1), hipMemcpyHostToDevice), "upload host offsets");
  hipCheck(hipMemcpy(dHBrk_, hBrk, sizeof(int32_t) * hOff[H], hipMemcpyHostToDevice), "upload host brokers");
}

ChainTables Device::chainTables() const {
  ChainTables c;
  c.brokers = brokers_;
  c.replicas = replicas_;
  c.parts = parts_;
  c.topicCount = topicCount_;
  c.topicLead = topicLead_;
  c.ldB = ldB_;
  c.W = W_;
  c.rLoad = dRLoad_;
  c.bLoad = dBLoad_;
  c.bLnw = dBLnw_;
  c.bPot = dBPot_;
  c.pOff = dPOff_;
  c.pSlots = dPSlots_;
  c.pLeader = dPLeader_;
  c.hLoad = dHLoad_;
  c.bHost = dBHost_;
  c.hOff = dHOff_;
  c.hBrk = dHBrk_;
  return c;
}

// [row updates | load rows | slot rows | request]; launches sync_loads and prep (rows applied, request copied into
// HBM at dReq_). `fill` writes the request into the staging area.
template <class F>
size_t Device::stageChainCopy(size_t reqBytes, Staged& g, size_t& oReq, F fill, void* stream) {
  if (!dRLoad_) throw std::runtime_error("device chain state not uploaded");
  const size_t nl = lrows.size(), ns = srows.size();
  const size_t oL = 0, oS = align16(nl * sizeof(LoadRow)), oR = oS + align16(ns * sizeof(SlotRow));
  g = packUpdates(oR + reqBytes);
  std::memcpy(hStage_ + g.end + oL, lrows.data(), nl * sizeof(LoadRow));
  std::memcpy(hStage_ + g.end + oS, srows.data(), ns * sizeof(SlotRow));
  fill(hStage_ + g.end + oR);
  hipCheck(launchSyncLoads(chainTables(), (const LoadRow*)(hStageDev_ + g.end + oL), (int)nl,
                           (const SlotRow*)(hStageDev_ + g.end + oS), (int)ns, (hipStream_t)stream),
           "sync_loads");
  lrows.clear();
  srows.clear();
  // prep copies [g.end + oR, + reqBytes) into dReq_ when given the request at that offset
  Staged h = g;
  h.end = g.end + oR;
  launchPrepFor(h, reqBytes, false);
  (void)stream;
  oReq = 0;
  return g.end + oR;
}

void Device::ensureChainLog(size_t n) {
  if (n <= chainLogCap_) return;
  if (hChainLog_) (void)hipHostFree(hChainLog_);
  hChainLog_ = hChainLogDev_ = nullptr;
  chainLogCap_ = std::max<size_t>(n * 2, 4096);
  hipCheck(hipHostMalloc((void**)&hChainLog_, chainLogCap_ * sizeof(int32_t), hipHostMallocMapped | hipHostMallocCoherent),
           "hipHostMalloc chain log");
  hipCheck(hipHostGetDevicePointer((void**)&hChainLogDev_, hChainLog_, 0), "hipHostGetDevicePointer");
}

Device::ChainResult Device::chainPairs(const DevProgram& prog, const int32_t* pr, const int32_t* pb,
                                       const int32_t* next, int n, int maxAccepts, std::vector<int32_t>& log) {
  DeviceGuard dg(ordinal_);
  ChainResult res;
  log.clear();
  if (n <= 0) {
    flushPending();
    return res;
  }
  ensureChainLog((size_t)n);
  // the running server takes the chain as a command (no stop and relaunch around it); otherwise one launch
  const auto tw = prof().on ? std::chrono::steady_clock::now() : std::chrono::steady_clock::time_point();
  const bool served = serverChain(prog, CM_PAIRS, pr, n, pb, n, next, n, n, 0, maxAccepts);
  if (prof().on) {
    prof().count(36, "chain.ns.command",
                 (int64_t)std::chrono::duration_cast<std::chrono::nanoseconds>(std::chrono::steady_clock::now() - tw)
                     .count());
    prof().count(37, "chain.lrows", (int64_t)lrowsSent_);
    prof().count(38, "chain.srows", (int64_t)srowsSent_);
  }
  if (!served) {
    stopServer();
    const size_t oB = align16((size_t)n * sizeof(RowRef)), oN = oB + align16((size_t)n * 4),
                 req = oN + align16((size_t)n * 4);
    Staged g;
    size_t oReq = 0;
    (void)stageChainCopy(req, g, oReq, [&](char* base) {
      writeRowRefs(base, pr, (size_t)n);
      std::memcpy(base + oB, pb, (size_t)n * 4);
      std::memcpy(base + oN, next, (size_t)n * 4);
    }, st_);
    if (timing) (void)hipEventRecord(EV0, ST);
    hipCheck(launchChainPairs(tables(), chainTables(), prog, (const RowRef*)dReq_, (const int32_t*)(dReq_ + oB),
                              (const int32_t*)(dReq_ + oN), n, maxAccepts, hChainLogDev_, hChainOutDev_, ST),
             "chain_pairs");
    if (timing) (void)hipEventRecord(EV1, ST);
    streamWait("chain_pairs", kChainWaitSeconds);
    perf.scanLaunches++;
    perf.chainLaunches++;
    if (timing) {
      float ms = 0.f;
      hipCheck(hipEventElapsedTime(&ms, EV0, EV1), "hipEventElapsedTime");
      perf.scanKernelMs += ms;
    }
  }
  const volatile ChainResultDev* vo = hChainOut_;
  const ChainResultDev out{vo->accepts, vo->visited, vo->failRow};
  perf.syncs++;
  perf.scanPairs += (int64_t)out.visited;
  perf.scanRequired += (int64_t)out.visited;
  res.accepts = (int64_t)out.accepts;
  res.visited = (int64_t)out.visited;
  log.resize((size_t)res.accepts);
  if (res.accepts) std::memcpy(log.data(), hChainLog_, sizeof(int32_t) * res.accepts);
  return res;
}

int64_t Device::rackRowsGroups(const DevProgram& prog, const int32_t* rows, int n, const int32_t* order,
                               const int32_t* gOff, int G, const int32_t* cands, int N, int32_t* res) {
  DeviceGuard dg(ordinal_);
  stopServer();
  if (n <= 0 || G <= 0) {
    flushPending();
    return 0;
  }
  // request [rows | order | gOff | cands] into HBM with the pending rows (prep), then one lane per partition group
  const size_t oO = align16((size_t)n * 4), oG = oO + align16((size_t)n * 4), oC = oG + align16((size_t)(G + 1) * 4);
  const size_t req = oC + align16((size_t)N * 4);
  const Staged g = packUpdates(req);
  std::memcpy(hStage_ + g.end, rows, (size_t)n * 4);
  std::memcpy(hStage_ + g.end + oO, order, (size_t)n * 4);
  std::memcpy(hStage_ + g.end + oG, gOff, (size_t)(G + 1) * 4);
  std::memcpy(hStage_ + g.end + oC, cands, (size_t)N * 4);
  launchPrepFor(g, req, false);
  if ((size_t)n > rackResCap_) {
    if (dRackRes_) hipCheck(hipFree(dRackRes_), "hipFree");
    rackResCap_ = (size_t)n * 2;
    hipCheck(hipMalloc((void**)&dRackRes_, rackResCap_ * 4 + 16), "hipMalloc rack rows");
  }
  unsigned long long* dEval = reinterpret_cast<unsigned long long*>(dRackRes_ + rackResCap_);
  hipCheck(hipMemsetAsync(dEval, 0, sizeof(unsigned long long), ST), "memset");
  if (timing) (void)hipEventRecord(EV0, ST);
  hipCheck(launchRackRowsGroups(tables(), prog, (const int32_t*)dReq_, (const int32_t*)(dReq_ + oO),
                                (const int32_t*)(dReq_ + oG), G, (const int32_t*)(dReq_ + oC), N, dRackRes_, dEval, ST),
           "rack_rows_groups");
  if (timing) (void)hipEventRecord(EV1, ST);
  unsigned long long evaluated = 0;
  hipCheck(hipMemcpyAsync(res, dRackRes_, (size_t)n * 4, hipMemcpyDeviceToHost, ST), "D2H rack rows");
  hipCheck(hipMemcpyAsync(&evaluated, dEval, sizeof(evaluated), hipMemcpyDeviceToHost, ST), "D2H rack rows");
  streamWait("rack_rows_groups", kChainWaitSeconds);
  perf.syncs++;
  perf.scanLaunches++;
  perf.scanPairs += (int64_t)evaluated;
  perf.scanRequired += (int64_t)evaluated;
  perf.scanBytes += (int64_t)evaluated * kBytesPerCandidate;
  if (timing) {
    float ms = 0.f;
    hipCheck(hipEventElapsedTime(&ms, EV0, EV1), "hipEventElapsedTime");
    perf.scanKernelMs += ms;
  }
  return (int64_t)evaluated;
}

Device::ChainResult Device::chainRackRows(const DevProgram& prog, const int32_t* rows, int n, const int32_t* cands,
                                          int N, std::vector<int32_t>& log) {
  DeviceGuard dg(ordinal_);
  ChainResult res;
  log.clear();
  if (n <= 0) {
    flushPending();
    return res;
  }
  ensureChainLog((size_t)2 * n);
  const bool served = serverChain(prog, CM_RACK_ROWS, rows, n, cands, N, nullptr, 0, n, N, 0);
  if (!served) {
    stopServer();
    const size_t oC = align16((size_t)n * 4), req = oC + align16((size_t)N * 4);
    Staged g;
    size_t oReq = 0;
    (void)stageChainCopy(req, g, oReq, [&](char* base) {
      std::memcpy(base, rows, (size_t)n * 4);
      std::memcpy(base + oC, cands, (size_t)N * 4);
    }, st_);
    if (timing) (void)hipEventRecord(EV0, ST);
    hipCheck(launchChainRackRows(tables(), chainTables(), prog, (const int32_t*)dReq_, n,
                                 (const int32_t*)(dReq_ + oC), N, hChainLogDev_, hChainOutDev_, ST),
             "chain_rack_rows");
    if (timing) (void)hipEventRecord(EV1, ST);
    streamWait("chain_rack_rows", kChainWaitSeconds);
    perf.scanLaunches++;
    perf.chainLaunches++;
    if (timing) {
      float ms = 0.f;
      hipCheck(hipEventElapsedTime(&ms, EV0, EV1), "hipEventElapsedTime");
      perf.scanKernelMs += ms;
    }
  }
  const volatile ChainResultDev* vo = hChainOut_;
  const ChainResultDev out{vo->accepts, vo->visited, vo->failRow};
  perf.syncs++;
  res.accepts = (int64_t)out.accepts;
  res.failRow = (int64_t)out.failRow;
  log.resize((size_t)res.accepts * 2);
  if (res.accepts) std::memcpy(log.data(), hChainLog_, sizeof(int32_t) * 2 * res.accepts);
  int64_t evaluated = res.failRow ? N : 0;
  for (size_t i = 1; i < log.size(); i += 2) evaluated += log[i] + 1;
  perf.scanPairs += evaluated;
  perf.scanRequired += evaluated;
  return res;
}

}  // namespace ccmi

namespace ccmi {

// ------------------------------------------------------------------------------------------------ K6 intra-broker
namespace {
template <class T>
void dallocTracked(T** p, size_t n, std::vector<void*>& owned) {
  if (*p) {
    for (auto& q : owned)
      if (q == (void*)*p) q = nullptr;
    (void)hipFree(*p);
  }
  hipCheck(hipMalloc((void**)p, (n ? n : 1) * sizeof(T)), "hipMalloc");
  owned.push_back((void*)*p);
}
// grow three int32 device arrays sharing one capacity to n elements, keeping their first `keep` elements
void growTriple(int32_t** a, int32_t** b, int32_t** c, size_t& cap, size_t n, size_t keep, std::vector<void*>& owned,
                hipStream_t st) {
  if (n <= cap && *a) return;
  size_t nc = cap ? cap : 1024;
  while (nc < n) nc *= 2;
  int32_t** arrs[3] = {a, b, c};
  for (int32_t** p : arrs) {
    int32_t* q = nullptr;
    hipCheck(hipMalloc((void**)&q, nc * sizeof(int32_t)), "hipMalloc");
    if (*p && keep) hipCheck(hipMemcpyAsync(q, *p, keep * sizeof(int32_t), hipMemcpyDeviceToDevice, st), "grow copy");
    if (*p) {
      hipCheck(hipStreamSynchronize(st), "sync");
      for (auto& x : owned)
        if (x == (void*)*p) x = nullptr;
      (void)hipFree(*p);
    }
    owned.push_back((void*)q);
    *p = q;
  }
  cap = nc;
}
}  // namespace

void Device::uploadDisks(int D, const int32_t* bDiskOff, const int32_t* bDisks, const double* dCap,
                         const uint8_t* dAlive, const uint8_t* bAlive, const int32_t* rOrigDisk, const double* rDu,
                         const float* rScore, const int32_t* rTie) {
  DeviceGuard dg(ordinal_);
  stopServer();
  D_ = D;
  auto& o = intraAllocs_;
  dallocTracked(&dBDiskOff_, (size_t)B_ + 1, o);
  dallocTracked(&dBDisks_, (size_t)D, o);
  dallocTracked(&dDCap_, (size_t)D, o);
  dallocTracked(&dDAlive_, (size_t)D, o);
  dallocTracked(&dDUtilIn_, (size_t)D, o);
  dallocTracked(&dDUtil_, (size_t)D, o);
  dallocTracked(&dBAlive_, (size_t)B_, o);
  dallocTracked(&dROrigDisk_, (size_t)R_, o);
  dallocTracked(&dRDu_, (size_t)R_, o);
  dallocTracked(&dRScore_, (size_t)R_, o);
  dallocTracked(&dRTie_, (size_t)R_, o);
  dallocTracked(&dRSel_, (size_t)R_, o);
  dallocTracked(&dUpper_, (size_t)G_ * B_, o);
  dallocTracked(&dLower_, (size_t)G_ * B_, o);
  dallocTracked(&dHist_, (size_t)B_ * kIntraHist * (kIntraMaxDisks + 1), o);
  dallocTracked(&dBrokers_, (size_t)B_, o);
  dallocTracked(&dLogCap_, (size_t)B_, o);
  dallocTracked(&dCount_, (size_t)B_, o);
  dallocTracked(&dStatus_, (size_t)B_, o);
  dallocTracked(&dLogOff_, (size_t)B_, o);
  dallocTracked(&dCand_, (size_t)B_, o);
  dallocTracked(&dCOff_, (size_t)B_ + 1, o);
  dallocTracked(&dEOff_, (size_t)B_ + 1, o);
  dallocTracked(&dNSel_, (size_t)B_, o);
  dallocTracked(&dDiskStats_, 1 + kDiskStatsBlocks, o);
  hipCheck(hipMemcpy(dBDiskOff_, bDiskOff, sizeof(int32_t) * (B_ + 1), hipMemcpyHostToDevice), "upload bDiskOff");
  hipCheck(hipMemcpy(dBDisks_, bDisks, sizeof(int32_t) * D, hipMemcpyHostToDevice), "upload bDisks");
  hipCheck(hipMemcpy(dDCap_, dCap, sizeof(double) * D, hipMemcpyHostToDevice), "upload dCap");
  hipCheck(hipMemcpy(dDAlive_, dAlive, D, hipMemcpyHostToDevice), "upload dAlive");
  hipCheck(hipMemcpy(dBAlive_, bAlive, B_, hipMemcpyHostToDevice), "upload bAlive");
  hipCheck(hipMemcpy(dROrigDisk_, rOrigDisk, sizeof(int32_t) * R_, hipMemcpyHostToDevice), "upload rOrigDisk");
  hipCheck(hipMemcpy(dRDu_, rDu, sizeof(double) * R_, hipMemcpyHostToDevice), "upload rDu");
  hipCheck(hipMemcpy(dRScore_, rScore, sizeof(float) * R_, hipMemcpyHostToDevice), "upload rScore");
  hipCheck(hipMemcpy(dRTie_, rTie, sizeof(int32_t) * R_, hipMemcpyHostToDevice), "upload rTie");
  {
    std::vector<IntraRep> st((size_t)R_);
    for (int r = 0; r < R_; ++r) st[r] = IntraRep{rDu[r], rScore[r], rTie[r], rOrigDisk[r], {0, 0, 0}};
    dallocTracked(&dRStat_, (size_t)R_, o);
    hipCheck(hipMemcpy(dRStat_, st.data(), sizeof(IntraRep) * R_, hipMemcpyHostToDevice), "upload replica records");
  }
  hBDiskOff_.assign(bDiskOff, bDiskOff + B_ + 1);
}

void Device::setDiskUtil(const double* dUtil) {
  DeviceGuard dg(ordinal_);
  stopServer();
  hipCheck(hipMemcpyAsync(dDUtilIn_, dUtil, sizeof(double) * D_, hipMemcpyHostToDevice, ST), "upload dUtil");
}

void Device::intraRun(const IntraRequest& q, IntraResult& out) {
  DeviceGuard dg(ordinal_);
  stopServer();
  if (!dBDiskOff_) throw std::runtime_error("intraRun before uploadDisks");
  const size_t E = (size_t)q.eOff[B_];
  auto& o = intraAllocs_;
  if (E > entCap_ || !dERep_) {
    size_t c = 1024;
    while (c < E) c *= 2;
    dallocTracked(&dERep_, c, o);
    dallocTracked(&dEDiskIn_, c, o);
    dallocTracked(&dEDisk_, c, o);
    dallocTracked(&dSnapA_, c, o);
    dallocTracked(&dSnapB_, c, o);
    dallocTracked(&dOrdRev_, c, o);
    dallocTracked(&dOrdFwd_, c, o);
    dallocTracked(&dEDu_, c, o);
    dallocTracked(&dEOrig_, c, o);
    dallocTracked(&dEKeyRev_, c, o);
    dallocTracked(&dEKeyFwd_, c, o);
    entCap_ = c;
  }
  hipCheck(hipMemcpyAsync(dEOff_, q.eOff, sizeof(int32_t) * (B_ + 1), hipMemcpyHostToDevice, ST), "eOff");
  hipCheck(hipMemcpyAsync(dERep_, q.eRep, sizeof(int32_t) * E, hipMemcpyHostToDevice, ST), "eRep");
  hipCheck(hipMemcpyAsync(dEDiskIn_, q.eDisk, sizeof(int32_t) * E, hipMemcpyHostToDevice, ST), "eDisk");
  hipCheck(hipMemcpyAsync(dRSel_, q.rSel, R_, hipMemcpyHostToDevice, ST), "rSel");
  hipCheck(hipMemcpyAsync(dBrokers_, q.brokers, sizeof(int32_t) * q.nBrokers, hipMemcpyHostToDevice, ST), "brokers");
  hipCheck(hipMemsetAsync(dCount_, 0, sizeof(int32_t) * B_, ST), "memset");
  hipCheck(hipMemsetAsync(dStatus_, 0, sizeof(int32_t) * B_, ST), "memset");
  hipCheck(hipMemsetAsync(dCand_, 0, sizeof(int64_t) * B_, ST), "memset");
  // log ranges: 2 records per replica + 64 first; a broker that runs out is re-run with the bound of its program
  std::vector<int64_t> logOff(B_, 0);
  std::vector<int32_t> cap(B_, 0);
  int64_t total = 0;
  for (int i = 0; i < q.nBrokers; ++i) {
    const int b = q.brokers[i];
    logOff[b] = total;
    cap[b] = 2 * (q.eOff[b + 1] - q.eOff[b]) + 64;
    total += cap[b];
  }
  growTriple(&dLogRep_, &dLogSrc_, &dLogDst_, logCap_, (size_t)total, 0, o, ST);
  IntraArgs A{};
  A.goal = q.goal;
  A.capThr = q.capThr;
  A.margin = q.margin;
  A.nPrior = q.nPrior;
  if (q.nPrior > kIntraMaxPrior) throw std::invalid_argument("too many optimized intra-broker goals");
  for (int k = 0; k < q.nPrior; ++k) {
    A.prior[k].kind = q.priorKind[k];
    A.prior[k].upper = dUpper_ + (size_t)q.priorSlot[k] * B_;
    A.prior[k].lower = dLower_ + (size_t)q.priorSlot[k] * B_;
  }
  A.brokers = dBrokers_;
  A.nBrokers = q.nBrokers;
  A.bDiskOff = dBDiskOff_;
  A.bDisks = dBDisks_;
  A.dCap = dDCap_;
  A.dAlive = dDAlive_;
  A.dUtilIn = dDUtilIn_;
  A.dUtil = dDUtil_;
  A.eOff = dEOff_;
  A.eRep = dERep_;
  A.eDiskIn = dEDiskIn_;
  A.eDisk = dEDisk_;
  A.rDu = dRDu_;
  A.rScore = dRScore_;
  A.rTie = dRTie_;
  A.rOrigDisk = dROrigDisk_;
  A.rStat = dRStat_;
  A.rSel = dRSel_;
  A.snapA = dSnapA_;
  A.snapB = dSnapB_;
  A.ordRev = dOrdRev_;
  A.ordFwd = dOrdFwd_;
  A.eDu = dEDu_;
  A.eOrig = dEOrig_;
  A.eKeyRev = dEKeyRev_;
  A.eKeyFwd = dEKeyFwd_;
  A.nSel = dNSel_;
  A.hist = dHist_;
  A.upperOut = dUpper_ + (size_t)q.slot * B_;
  A.lowerOut = dLower_ + (size_t)q.slot * B_;
  A.logOff = dLogOff_;
  A.logCap = dLogCap_;
  A.logRep = dLogRep_;
  A.logSrc = dLogSrc_;
  A.logDst = dLogDst_;
  A.logCount = dCount_;
  A.status = dStatus_;
  A.cand = dCand_;
  float msTotal = 0.f;
  bool sorted = false;
  auto launch = [&](const IntraArgs& a) {
    hipCheck(hipMemcpyAsync(dLogOff_, logOff.data(), sizeof(int64_t) * B_, hipMemcpyHostToDevice, ST), "logOff");
    hipCheck(hipMemcpyAsync(dLogCap_, cap.data(), sizeof(int32_t) * B_, hipMemcpyHostToDevice, ST), "logCap");
    // kernel timing: intra_sort (once per call) and intra_brokers bracketed separately, so the K6 headline is
    // intra_brokers alone (the kernel its algorithmic bytes count; rocprofv3 reports the two apart)
    const bool sortNow = !sorted;
    if (timing) hipCheck(hipEventRecord(EV2, ST), "event");
    if (sortNow) hipCheck(launchIntraSort(a, ST), "intra_sort");
    sorted = true;
    if (timing) hipCheck(hipEventRecord(EV0, ST), "event");
    hipCheck(launchIntra(a, ST), "intra_brokers");
    if (timing) hipCheck(hipEventRecord(EV1, ST), "event");
    out.status.resize(B_);
    hipCheck(hipMemcpyAsync(out.status.data(), dStatus_, sizeof(int32_t) * B_, hipMemcpyDeviceToHost, ST), "status");
    hipCheck(hipStreamSynchronize(ST), "intra sync");
    perf.syncs++;
    perf.intraLaunches++;
    if (timing) {
      float ms = 0.f;
      hipCheck(hipEventElapsedTime(&ms, EV0, EV1), "hipEventElapsedTime");
      msTotal += ms;
      if (sortNow) {
        hipCheck(hipEventElapsedTime(&ms, EV2, EV0), "hipEventElapsedTime");
        perf.intraSortMs += ms;
        perf.intraSorts++;
      }
    }
  };
  launch(A);
  std::vector<int32_t> rerun;
  for (int i = 0; i < q.nBrokers; ++i)
    if (out.status[q.brokers[i]] == IS_LOG_FULL) rerun.push_back(q.brokers[i]);
  if (!rerun.empty()) {
    const int64_t keep = total;
    for (int b : rerun) {
      const int64_t n = q.eOff[b + 1] - q.eOff[b];
      const int64_t nd = hBDiskOff_[b + 1] - hBDiskOff_[b];
      logOff[b] = total;
      cap[b] = (int32_t)(6 * (nd + 1) * n + 64);
      total += cap[b];
    }
    growTriple(&dLogRep_, &dLogSrc_, &dLogDst_, logCap_, (size_t)total, (size_t)keep, o, ST);
    A.logRep = dLogRep_;
    A.logSrc = dLogSrc_;
    A.logDst = dLogDst_;
    hipCheck(hipMemcpyAsync(dBrokers_, rerun.data(), sizeof(int32_t) * rerun.size(), hipMemcpyHostToDevice, ST),
             "rerun brokers");
    A.nBrokers = (int)rerun.size();
    launch(A);
    for (int b : rerun)
      if (out.status[b] == IS_LOG_FULL) throw std::runtime_error("device intra-broker log overflow");
    hipCheck(hipMemcpyAsync(dBrokers_, q.brokers, sizeof(int32_t) * q.nBrokers, hipMemcpyHostToDevice, ST), "brokers");
  }
  perf.intraKernelMs += msTotal;
  out.count.resize(B_);
  out.cand.resize(B_);
  hipCheck(hipMemcpyAsync(out.count.data(), dCount_, sizeof(int32_t) * B_, hipMemcpyDeviceToHost, ST), "count");
  hipCheck(hipMemcpyAsync(out.cand.data(), dCand_, sizeof(int64_t) * B_, hipMemcpyDeviceToHost, ST), "cand");
  hipCheck(hipStreamSynchronize(ST), "intra sync");
  out.off.assign(B_ + 1, 0);
  for (int b = 0; b < B_; ++b) out.off[b + 1] = out.off[b] + out.count[b];
  const size_t nrec = (size_t)out.off[B_];
  growTriple(&dCRep_, &dCSrc_, &dCDst_, compactCap_, nrec, 0, o, ST);
  hipCheck(hipMemcpyAsync(dCOff_, out.off.data(), sizeof(int64_t) * (B_ + 1), hipMemcpyHostToDevice, ST), "cOff");
  hipCheck(hipMemcpyAsync(dLogOff_, logOff.data(), sizeof(int64_t) * B_, hipMemcpyHostToDevice, ST), "logOff");
  hipCheck(launchIntraCompact(dBrokers_, q.nBrokers, dLogOff_, dCount_, dCOff_, dLogRep_, dLogSrc_, dLogDst_, dCRep_,
                              dCSrc_, dCDst_, ST),
           "intra_compact");
  out.rep.resize(nrec);
  out.src.resize(nrec);
  out.dst.resize(nrec);
  if (nrec) {
    hipCheck(hipMemcpyAsync(out.rep.data(), dCRep_, sizeof(int32_t) * nrec, hipMemcpyDeviceToHost, ST), "rep");
    hipCheck(hipMemcpyAsync(out.src.data(), dCSrc_, sizeof(int32_t) * nrec, hipMemcpyDeviceToHost, ST), "src");
    hipCheck(hipMemcpyAsync(out.dst.data(), dCDst_, sizeof(int32_t) * nrec, hipMemcpyDeviceToHost, ST), "dst");
  }
  if (q.goal == IG_USAGE) {
    out.upper.resize(B_);
    out.lower.resize(B_);
    hipCheck(hipMemcpyAsync(out.upper.data(), dUpper_ + (size_t)q.slot * B_, sizeof(double) * B_,
                            hipMemcpyDeviceToHost, ST), "upper");
    hipCheck(hipMemcpyAsync(out.lower.data(), dLower_ + (size_t)q.slot * B_, sizeof(double) * B_,
                            hipMemcpyDeviceToHost, ST), "lower");
  }
  hipCheck(hipStreamSynchronize(ST), "intra sync");
  perf.syncs++;
  // algorithmic bytes: every processed broker's disk records and replica entries read once
  int64_t bytes = 0;
  for (int i = 0; i < q.nBrokers; ++i) {
    const int b = q.brokers[i];
    bytes += (int64_t)(hBDiskOff_[b + 1] - hBDiskOff_[b]) * kIntraBytesPerDisk +
             (int64_t)(q.eOff[b + 1] - q.eOff[b]) * kIntraBytesPerEntry;
  }
  perf.intraBytes += bytes;
}

void Device::statsDisks(double diskBalance, DiskStatsOut* out) {
  DeviceGuard dg(ordinal_);
  stopServer();
  hipCheck(launchStatsDisks(dBDiskOff_, dBDisks_, dDCap_, dDAlive_, dDUtilIn_, dBAlive_, B_, diskBalance, dDiskStats_,
                            ST),
           "stats_disks");
  hipCheck(hipMemcpyAsync(out, dDiskStats_, sizeof(DiskStatsOut), hipMemcpyDeviceToHost, ST), "disk stats");
  hipCheck(hipStreamSynchronize(ST), "sync");
  perf.syncs++;
}

}  // namespace ccmi
