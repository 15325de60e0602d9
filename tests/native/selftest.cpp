// Standalone native self-test (no Python): exercises every threaded component
// concurrently so ASan/UBSan and TSan builds can check them (the
// reference never ran a race detector and has real races, e.g. the `restart` bool).
//
//   python -m k8s_gpu_device_plugin_amd._build --selftest            (plain)
//   python -m k8s_gpu_device_plugin_amd._build --sanitize address    (ASan + UBSan)
//   python -m k8s_gpu_device_plugin_amd._build --sanitize thread     (TSan)
#include <arpa/inet.h>
#include <netinet/in.h>
#include <sys/socket.h>
#include <unistd.h>

#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <memory>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

#include "allocator.h"
#include "device_table.h"
#include "fixture_backend.h"
#include "grpc_h2.h"
#include "health.h"
#include "hpack.h"
#include "httpd.h"
#include "pbwire.h"
#include "telemetry.h"

using namespace amdgpu_dp;

static int g_failures = 0;
#define CHECK(cond)                                                      \
  do {                                                                   \
    if (!(cond)) {                                                       \
      std::fprintf(stderr, "CHECK failed %s:%d: %s\n", __FILE__, __LINE__, #cond); \
      ++g_failures;                                                      \
    }                                                                    \
  } while (0)

static std::shared_ptr<FixtureBackend> make_node(int ngpu, int nparts) {
  auto be = std::make_shared<FixtureBackend>(7);
  int render = 128;
  for (int g = 0; g < ngpu; ++g) {
    GpuInfo gi;
    gi.uuid = "gpu-" + std::to_string(g);
    gi.market_name = "AMD Instinct MI355X";
    gi.gfx_target = "gfx950";
    gi.numa_node = g / 4;
    gi.vram_total_bytes = 288ull * 1000000000ull;
    gi.compute_partition = nparts == 1 ? "SPX" : "CPX";
    gi.memory_partition = "NPS1";
    for (int p = 0; p < nparts; ++p) {
      PartitionInfo pi;
      pi.id = gi.uuid + "-xcp" + std::to_string(p);
      pi.index = p;
      pi.render_minor = render++;
      pi.numa_node = gi.numa_node;
      gi.partitions.push_back(pi);
    }
    be->add_gpu(gi);
  }
  for (int a = 0; a < ngpu; ++a)
    for (int b = a + 1; b < ngpu; ++b) {
      Link l;
      l.type = kLinkXgmi;
      l.hops = 1;
      be->set_link(a, b, l);
    }
  return be;
}

static std::string alloc_req(const std::string& id) {
  std::string c, r;
  pb::put_bytes(&c, 1, id);
  pb::put_bytes(&r, 1, c);
  return r;
}

static void test_hpack() {
  std::string enc, dec;
  hpack::huffman_encode("www.example.com", &enc);
  CHECK(hpack::huffman_decode(reinterpret_cast<const uint8_t*>(enc.data()), enc.size(), &dec));
  CHECK(dec == "www.example.com");
  hpack::Decoder d;
  std::string block;
  hpack::encode_indexed(&block, 3);
  hpack::encode_literal(&block, "te", "trailers", true);
  std::vector<hpack::Header> hs;
  CHECK(d.decode(reinterpret_cast<const uint8_t*>(block.data()), block.size(), &hs));
  CHECK(hs.size() == 2 && hs[0].value == "POST" && hs[1].value == "trailers");
}

static void test_allocator_and_table(std::shared_ptr<FixtureBackend> be) {
  std::vector<GpuInfo> gpus;
  Topology topo;
  be->discover(&gpus, &topo);
  std::vector<TableDevice> devs;
  for (auto& g : gpus)
    for (auto& p : g.partitions) {
      TableDevice d;
      d.id = p.id;
      d.gpu = g.index;
      d.partition = p.index;
      d.numa = p.numa_node;
      d.host_paths = {"/dev/dri/renderD" + std::to_string(p.render_minor)};
      devs.push_back(d);
    }
  auto table = std::make_shared<DeviceTable>(TableConfig{}, devs, topo);
  std::string out;
  CHECK(table->allocate(alloc_req(devs[3].id), &out));
  CHECK(!table->allocate(alloc_req("nope"), &out));
  std::vector<std::string> ids;
  AllocResult r = table->preferred_ids(table->ids(), {}, 8, &ids);
  CHECK(r.ok && ids.size() == 8);
  // concurrent readers + health writers
  std::atomic<bool> stop{false};
  std::vector<std::thread> ts;
  for (int i = 0; i < 4; ++i)
    ts.emplace_back([&, i] {
      std::string o;
      std::vector<std::string> got;
      while (!stop.load()) {
        table->allocate(alloc_req(devs[i].id), &o);
        table->list_and_watch();
        table->preferred_ids(table->ids(), {}, 2, &got);
      }
    });
  for (int k = 0; k < 200; ++k) table->set_gpu_health(k % 8, -1, k % 2);
  stop = true;
  for (auto& t : ts) t.join();
}

static void test_grpc_server(std::shared_ptr<FixtureBackend> be, const std::string& dir) {
  std::vector<GpuInfo> gpus;
  Topology topo;
  be->discover(&gpus, &topo);
  std::vector<TableDevice> devs;
  for (auto& g : gpus) {
    TableDevice d;
    d.id = g.uuid;
    d.gpu = g.index;
    d.numa = g.numa_node;
    devs.push_back(d);
  }
  TableConfig tc;
  tc.reject_unhealthy = false;  // health flips concurrently below
  auto table = std::make_shared<DeviceTable>(tc, devs, topo);
  const std::string path = dir + "/selftest.sock";
  GrpcServer srv(path, 3);
  srv.set_table(table);
  srv.start();
  std::atomic<int> errors{0};
  std::vector<std::thread> ts;
  for (int i = 0; i < 6; ++i)
    ts.emplace_back([&, i] {
      try {
        H2Client c(path);
        std::string resp, msg;
        for (int k = 0; k < 300; ++k)
          if (c.unary("/v1beta1.DevicePlugin/Allocate", alloc_req(devs[i % devs.size()].id), &resp, &msg) != 0)
            ++errors;
        std::string law;
        c.first_stream_message("/v1beta1.DevicePlugin/ListAndWatch", "", &law);
        if (law.empty()) ++errors;
      } catch (const std::exception& e) {
        std::fprintf(stderr, "client error: %s\n", e.what());
        ++errors;
      }
    });
  // the monitor thread's fail-fast path pushes through the table listener while the
  // main thread also flips health and clients call in
  auto mon = std::make_shared<HealthMonitor>(be, 2);
  mon->set_gpu_count(static_cast<int>(gpus.size()));
  mon->set_fast_tables({table});
  mon->start();
  for (int k = 0; k < 50; ++k) {
    table->set_gpu_health(k % 4, -1, k % 2);
    srv.notify();
    HwEvent e;
    e.kind = k % 2 ? kEvtPostReset : kEvtPreReset;
    e.gpu = k % 4;
    be->inject_event(e);
  }
  for (auto& t : ts) t.join();
  mon->stop();
  CHECK(errors.load() == 0);
  CHECK(srv.requests() >= 1800);
  srv.stop();
  srv.stop();
}

// Plugin reloads racing health transitions: an event thread flips GPUs while the main
// thread keeps attaching fresh tables.  After every attach the newest table must agree
// with the monitor once the event thread pauses (no transition lost in the hand-over).
static void test_attach_tables_during_events(std::shared_ptr<FixtureBackend> be) {
  std::vector<GpuInfo> gpus;
  Topology topo;
  be->discover(&gpus, &topo);
  std::vector<TableDevice> devs;
  for (const auto& g : gpus) {
    TableDevice d;
    d.id = "gpu" + std::to_string(g.index);
    d.gpu = g.index;
    devs.push_back(d);
  }
  TableConfig tc;
  auto mon = std::make_shared<HealthMonitor>(be, 2);
  mon->set_gpu_count(static_cast<int>(gpus.size()));
  mon->start();
  for (int round = 0; round < 20; ++round) {
    std::atomic<bool> go{true};
    std::thread ev([&, round] {
      for (int k = 0; go.load() || k < 64; ++k) {
        HwEvent e;
        e.kind = (k + round) % 3 ? kEvtPreReset : kEvtPostReset;
        e.gpu = (k * 7 + round) % static_cast<int>(gpus.size());
        mon->process(e);
      }
    });
    std::shared_ptr<DeviceTable> last;
    for (int k = 0; k < 8; ++k) {
      last = std::make_shared<DeviceTable>(tc, devs, topo);
      mon->attach_tables({last}, true, {});
    }
    go.store(false);
    ev.join();
    for (const auto& g : gpus) CHECK(last->healthy("gpu" + std::to_string(g.index)) == mon->gpu_healthy(g.index));
  }
  mon->pop(0);
  mon->stop();
}

// PreStartContainer answered asynchronously: a verifier thread completes jobs while
// clients call, some clients disconnect with checks in flight, and the server stops
// with jobs still queued (their completions must land in a queue that outlives it).
static void test_prestart_async(const std::string& dir) {
  TableConfig tc;
  tc.pre_start_required = true;
  std::vector<TableDevice> devs;
  for (int i = 0; i < 4; ++i) {
    TableDevice d;
    d.id = "dev" + std::to_string(i);
    d.gpu = i;
    devs.push_back(d);
  }
  Topology topo;
  topo.resize(4);
  auto table = std::make_shared<DeviceTable>(tc, devs, topo);
  const std::string path = dir + "/prestart.sock";
  auto srv = std::make_unique<GrpcServer>(path, 2);
  srv->set_table(table);
  srv->start();
  std::atomic<bool> stop{false};
  std::atomic<int> completed{0};
  std::thread verifier([&] {
    uint64_t n = 0;
    while (!stop.load())
      for (auto& j : table->pop_prestart(20)) {
        if (++n % 4 == 0) std::this_thread::sleep_for(std::chrono::milliseconds(1));
        table->complete_prestart(j.id, n % 5 != 0, n % 5 ? "" : "injected failure");
        ++completed;
      }
  });
  std::atomic<int> errors{0}, failed{0};
  std::vector<std::thread> ts;
  for (int i = 0; i < 4; ++i)
    ts.emplace_back([&, i] {
      try {
        for (int round = 0; round < 5; ++round) {
          H2Client c(path);
          std::string resp, msg;
          std::string req;
          pb::put_bytes(&req, 1, devs[i].id);
          for (int k = 0; k < 20; ++k) {
            const int st = c.unary("/v1beta1.DevicePlugin/PreStartContainer", req, &resp, &msg);
            if (st == 2) ++failed;
            else if (st != 0) ++errors;
          }
          if (round % 2) c.close();  // next round reconnects (fd numbers get reused)
        }
      } catch (const std::exception& e) {
        std::fprintf(stderr, "prestart client error: %s\n", e.what());
        ++errors;
      }
    });
  for (auto& t : ts) t.join();
  CHECK(errors.load() == 0);
  CHECK(failed.load() > 0 && failed.load() < 400);
  // jobs left queued at stop: the server goes away, completions still find their queue
  {
    H2Client c(path);
    std::string req;
    pb::put_bytes(&req, 1, devs[0].id);
    c.send_unary_nowait("/v1beta1.DevicePlugin/PreStartContainer", req);
  }
  srv->stop();
  srv.reset();
  stop.store(true);
  verifier.join();
  table->cancel_prestart("stopping");
  CHECK(table->prestart_pending() == 0);
}

static void test_exporter_httpd_health(std::shared_ptr<FixtureBackend> be) {
  std::vector<GpuInfo> gpus;
  Topology topo;
  be->discover(&gpus, &topo);
  auto ex = std::make_shared<Exporter>();
  ex->set_inventory(gpus);
  auto mon = std::make_shared<HealthMonitor>(be, 2);
  mon->set_gpu_count(static_cast<int>(gpus.size()));
  mon->start();
  ex->start(be, 5, mon);
  HttpConfig hc;
  hc.host = "127.0.0.1";
  hc.port = 0;
  hc.threads = 3;
  hc.access_log = false;
  HttpServer http(hc, ex);
  std::atomic<int> restarts{0};
  http.set_restart_hook([&] { ++restarts; });
  const int port = http.start();
  std::atomic<int> bad{0};
  std::vector<std::thread> ts;
  for (int i = 0; i < 4; ++i)
    ts.emplace_back([&, i] {
      for (int k = 0; k < 40; ++k) {
        const int fd = socket(AF_INET, SOCK_STREAM, 0);
        if (fd < 0) {
          ++bad;
          continue;
        }
        sockaddr_in a{};
        a.sin_family = AF_INET;
        a.sin_port = htons(static_cast<uint16_t>(port));
        a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
        if (connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) != 0) {
          ++bad;
          close(fd);
          continue;
        }
        const char* req = (k % 3 == 0) ? (k % 2 ? "GET /metrics HTTP/1.1\r\nAccept-Encoding: gzip\r\nConnection: close\r\n\r\n"
                                                : "GET /metrics HTTP/1.1\r\nConnection: close\r\n\r\n")
                                       : (i == 0 && k == 1 ? "GET /restart HTTP/1.1\r\nConnection: close\r\n\r\n"
                                                           : "GET /health HTTP/1.1\r\nConnection: close\r\n\r\n");
        (void)!write(fd, req, std::strlen(req));
        std::string resp;
        char buf[65536];
        ssize_t r;
        while ((r = read(fd, buf, sizeof(buf))) > 0) resp.append(buf, static_cast<size_t>(r));
        close(fd);
        if (resp.compare(0, 15, "HTTP/1.1 200 OK") != 0) ++bad;
      }
    });
  HwEvent e;
  e.kind = kEvtPreReset;
  e.gpu = 1;
  be->inject_event(e);
  be->set_ecc_uncorrectable(0, 5);
  for (auto& t : ts) t.join();
  CHECK(bad.load() == 0);
  CHECK(restarts.load() == 1);
  http.stop();
  ex->stop();
  mon->stop();
  bool saw_unhealthy = false;
  for (auto& u : mon->pop(10))
    if (u.healthy == 0) saw_unhealthy = true;
  CHECK(saw_unhealthy || !mon->gpu_healthy(1));
}

// A plugin reload (manager.load_plugins) swaps the exporter's inventory, partition
// labels and device tables while HTTP workers render /metrics (plain and gzip) and the
// sampler ticks; a server stop races open ListAndWatch streams.
static std::string http_get(int port, const char* req) {
  const int fd = socket(AF_INET, SOCK_STREAM, 0);
  if (fd < 0) return std::string();
  sockaddr_in a{};
  a.sin_family = AF_INET;
  a.sin_port = htons(static_cast<uint16_t>(port));
  a.sin_addr.s_addr = htonl(INADDR_LOOPBACK);
  std::string resp;
  if (connect(fd, reinterpret_cast<sockaddr*>(&a), sizeof(a)) == 0) {
    (void)!write(fd, req, std::strlen(req));
    char buf[65536];
    ssize_t r;
    while ((r = read(fd, buf, sizeof(buf))) > 0) resp.append(buf, static_cast<size_t>(r));
  }
  close(fd);
  return resp;
}

static std::shared_ptr<DeviceTable> table_of(const std::vector<GpuInfo>& gpus, const Topology& topo) {
  std::vector<TableDevice> devs;
  for (auto& g : gpus)
    for (auto& p : g.partitions) {
      TableDevice d;
      d.id = p.id;
      d.gpu = g.index;
      d.partition = p.index;
      devs.push_back(d);
    }
  return std::make_shared<DeviceTable>(TableConfig{}, devs, topo);
}

static void test_reload_races(const std::string& dir) {
  auto be_a = make_node(2, 1), be_b = make_node(4, 8);
  std::vector<GpuInfo> ga, gb;
  Topology ta, tb;
  be_a->discover(&ga, &ta);
  be_b->discover(&gb, &tb);
  auto ex = std::make_shared<Exporter>();
  ex->set_inventory(ga);
  ex->set_tables({table_of(ga, ta)});
  ex->start(be_a, 2, nullptr);
  HttpConfig hc;
  hc.host = "127.0.0.1";
  hc.port = 0;
  hc.threads = 3;
  hc.access_log = false;
  HttpServer http(hc, ex);
  const int port = http.start();
  std::atomic<bool> stop{false};
  std::atomic<int> bad{0};
  std::vector<std::thread> ts;
  for (int i = 0; i < 3; ++i)
    ts.emplace_back([&, i] {
      while (!stop.load()) {
        const std::string r = http_get(port, i % 2 ? "GET /metrics HTTP/1.1\r\nAccept-Encoding: gzip\r\nConnection: close\r\n\r\n"
                                                   : "GET /metrics HTTP/1.1\r\nConnection: close\r\n\r\n");
        if (r.compare(0, 15, "HTTP/1.1 200 OK") != 0) ++bad;
      }
    });
  for (int k = 0; k < 60; ++k) {  // reloads flip between a 2-GPU SPX and a 4-GPU CPX node
    const bool b = k % 2;
    std::vector<PartitionLabel> labels;
    for (auto& g : b ? gb : ga)
      for (auto& p : g.partitions) labels.push_back({g.index, p.index, p.id, "amd.com/gpu"});
    ex->set_inventory(b ? gb : ga);
    ex->set_partition_labels(labels);
    std::vector<std::shared_ptr<DeviceTable>> tables;
    tables.push_back(table_of(b ? gb : ga, b ? tb : ta));
    ex->set_tables(std::move(tables));
    ex->set_extra("# extra " + std::to_string(k) + "\n");
    std::this_thread::sleep_for(std::chrono::milliseconds(2));
  }
  stop = true;
  for (auto& t : ts) t.join();
  CHECK(bad.load() == 0);
  http.stop();
  ex->stop();

  // server stop with ListAndWatch streams open and clients still calling
  auto table = table_of(ga, ta);
  const std::string path = dir + "/reload.sock";
  for (int round = 0; round < 3; ++round) {
    GrpcServer srv(path, 2);
    srv.set_table(table);
    srv.start();
    std::atomic<bool> done{false};
    std::vector<std::thread> cs;
    for (int i = 0; i < 3; ++i)
      cs.emplace_back([&] {
        try {
          H2Client c(path, 2.0);
          std::string law;
          c.first_stream_message("/v1beta1.DevicePlugin/ListAndWatch", "", &law);
          std::string resp, msg;
          while (!done.load()) c.unary("/v1beta1.DevicePlugin/Allocate", alloc_req(ga[0].partitions[0].id), &resp, &msg);
        } catch (const std::exception&) {
          // the server going away mid-call is the point of this test
        }
      });
    // health flips (table -> server listener pushes) race the server's stop
    std::thread flipper([&] {
      for (int k = 0; !done.load(); ++k) table->set_gpu_health(k % 2, -1, k % 3 == 0);
    });
    std::this_thread::sleep_for(std::chrono::milliseconds(20));
    table->set_gpu_health(0, -1, round % 2);
    srv.notify();
    srv.stop();
    done = true;
    flipper.join();
    for (auto& t : cs) t.join();
  }
}

// Histogram render cache: a cached text is reused only while nothing was observed,
// never mixes name/label sets, and concurrent observe + render (scrapes on several
// HTTP workers) always ends at the exact final counts.
static void test_histogram_render_cache() {
  Histogram h(rpc_buckets());
  std::string a, b, c;
  h.render(&a, "x_seconds", "rpc=\"a\",");
  h.render(&b, "x_seconds", "rpc=\"a\",");
  CHECK(a == b);
  h.observe(3e-6);
  h.render(&c, "x_seconds", "rpc=\"a\",");
  CHECK(c != a && c.find("x_seconds_count{rpc=\"a\"} 1\n") != std::string::npos);
  std::string d;
  h.render(&d, "y_seconds", "");
  CHECK(d.find("y_seconds_count 1\n") != std::string::npos && d.find("x_seconds") == std::string::npos);
  std::string u;
  h.render_uncached(&u, "y_seconds", "");
  CHECK(u == d);
  std::atomic<bool> go{true};
  std::vector<std::thread> rs;
  for (int t = 0; t < 3; ++t)
    rs.emplace_back([&] {
      std::string o;
      while (go.load()) {
        o.clear();
        h.render(&o, "x_seconds", "rpc=\"a\",");
      }
    });
  std::thread w([&] {
    for (int i = 0; i < 20000; ++i) h.observe(1e-4);
  });
  w.join();
  go = false;
  for (auto& t : rs) t.join();
  std::string fin, ref;
  h.render(&fin, "x_seconds", "rpc=\"a\",");
  h.render_uncached(&ref, "x_seconds", "rpc=\"a\",");
  CHECK(fin == ref && fin.find("x_seconds_count{rpc=\"a\"} 20001\n") != std::string::npos);
}

// Lanes: a throwing call is caught on the lane (which keeps serving), a wedged lane
// refuses new work past the stall bound, a lane destroyed mid-call is detached and its
// call still completes; the session gate refuses an old session's calls and a close
// that a call inside outlasts fails and reopens the gate.
static void test_lanes_and_gate() {
  {
    Lane lane("gpu-a");
    auto bad = std::make_shared<LaneJob>("throws", [] { throw std::runtime_error("driver said no"); });
    int ran = 0;
    auto good = std::make_shared<LaneJob>("ok", [&ran] { ++ran; });
    CHECK(lane.post(bad, 0) && lane.post(good, 0));
    CHECK(bad->wait(2000) && good->wait(2000));
    CHECK(bad->failed() && bad->error() == "driver said no" && !bad->dropped());
    // a job is done before the lane books it as completed: give the lane a moment
    for (int i = 0; i < 200 && lane.state().completed < 2; ++i) std::this_thread::sleep_for(std::chrono::milliseconds(1));
    CHECK(!good->failed() && ran == 1 && lane.state().completed == 2);
  }
  std::atomic<bool> release{false};
  std::atomic<int> finished{0};
  {
    auto lane = std::make_unique<Lane>("gpu-b");
    auto stuck = std::make_shared<LaneJob>("stuck", [&] {
      while (!release.load()) std::this_thread::sleep_for(std::chrono::milliseconds(1));
      finished.fetch_add(1);
    });
    CHECK(lane->post(stuck, 0));
    std::this_thread::sleep_for(std::chrono::milliseconds(30));
    auto refused = std::make_shared<LaneJob>("later", [&] { finished.fetch_add(100); });
    CHECK(!lane->post(refused, 10 * 1000000LL) && refused->dropped());  // in flight > 10 ms
    auto queued = std::make_shared<LaneJob>("queued", [&] { finished.fetch_add(100); });
    CHECK(lane->post(queued, 0));  // no stall bound: queued behind the stuck call
    CHECK(lane->state().inflight_what == "stuck" && lane->state().queued == 1);
    lane.reset();  // must not wait for the stuck call
    CHECK(queued->dropped() && !stuck->done());
    release = true;
    CHECK(stuck->wait(2000) && finished.load() == 1);
  }
  SessionGate g;
  const uint64_t s1 = g.session();
  CHECK(g.enter(s1));
  CHECK(!g.close(20));  // a call is inside: the close gives up, the gate stays open
  CHECK(g.enter(s1));
  g.leave();
  g.leave();
  CHECK(g.active() == 0 && g.close(20));
  std::atomic<bool> entered{false};
  std::thread t([&] { entered = g.enter(0); });  // waits while the gate is closed
  std::this_thread::sleep_for(std::chrono::milliseconds(20));
  CHECK(!entered.load());
  const uint64_t s2 = g.reopen();
  t.join();
  CHECK(entered.load() && s2 == s1 + 1);
  g.leave();
  CHECK(!g.enter(s1));  // handles of the previous session are never used again
  CHECK(g.active() == 0);
}

// RecentAllocations: many writers wrap the 64-slot ring while readers snapshot it.
// Readers must always finish (no slot left odd by two writers) and only ever see masks
// that were written; once the writers stop, every slot is readable again.
static void test_recent_allocations_ring() {
  RecentAllocations ra;
  const int64_t t0 = 1'000'000'000LL;
  std::atomic<bool> go{true};
  std::atomic<long> bad{0}, reads{0};
  std::vector<std::thread> ws, rs;
  for (int w = 0; w < 6; ++w)
    ws.emplace_back([&, w] {
      const uint64_t m = (1ull << w) | (1ull << (w + 1));  // GPU pair (w, w+1)
      for (int i = 0; i < 40000; ++i) ra.record(m, t0 + i);
    });
  for (int r = 0; r < 3; ++r)
    rs.emplace_back([&] {
      std::vector<int> pods(64);
      while (go.load(std::memory_order_relaxed)) {
        std::fill(pods.begin(), pods.end(), 0);
        const int live = ra.add_link_pods(8, t0 + 1000, &pods);
        int pairs = 0;  // every live entry is exactly one adjacent pair
        for (int a = 0; a < 8; ++a)
          for (int b = a + 1; b < 8; ++b) {
            if (pods[a * 8 + b] && b != a + 1) bad.fetch_add(1);
            pairs += pods[a * 8 + b];
          }
        if (pairs != live) bad.fetch_add(1);
        reads.fetch_add(1);
      }
    });
  for (auto& t : ws) t.join();
  go = false;
  for (auto& t : rs) t.join();
  CHECK(bad.load() == 0);
  CHECK(reads.load() > 0);
  CHECK(ra.live(t0 + 40000) == RecentAllocations::kSlots);  // no slot stuck mid-write
}

int main() {
  char tmpl[] = "/tmp/amdgpu-selftest-XXXXXX";
  const char* dir = mkdtemp(tmpl);
  if (!dir) return 2;
  std::fprintf(stderr, "[selftest] hpack\n");
  test_hpack();
  std::fprintf(stderr, "[selftest] histogram render cache\n");
  test_histogram_render_cache();
  std::fprintf(stderr, "[selftest] lanes + session gate\n");
  test_lanes_and_gate();
  std::fprintf(stderr, "[selftest] recent allocations ring\n");
  test_recent_allocations_ring();
  std::fprintf(stderr, "[selftest] allocator + table\n");
  auto be = make_node(8, 8);
  test_allocator_and_table(be);
  std::fprintf(stderr, "[selftest] grpc server\n");
  test_grpc_server(make_node(4, 1), dir);
  std::fprintf(stderr, "[selftest] prestart async\n");
  test_prestart_async(dir);
  std::fprintf(stderr, "[selftest] exporter + httpd + health\n");
  test_exporter_httpd_health(make_node(2, 1));
  std::fprintf(stderr, "[selftest] reload races\n");
  test_reload_races(dir);
  std::fprintf(stderr, "[selftest] health hand-over on reload\n");
  test_attach_tables_during_events(make_node(4, 1));
  rmdir(dir);
  if (g_failures) {
    std::fprintf(stderr, "native selftest: %d failure(s)\n", g_failures);
    return 1;
  }
  std::printf("native selftest: ok\n");
  return 0;
}
