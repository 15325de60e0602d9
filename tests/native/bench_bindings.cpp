// pybind11 module `k8s_gpu_device_plugin_amd._native_bench`: the load generators and
// latency probes of bench.py, the BASELINE.md protocol, scripts/ and the tests.  None of
// it ships in the plugin's own extension (`_native`): a DaemonSet pod never loads it.
//
// It links the same core objects as `_native` and works on objects `_native` created
// (its H2Client, Exporter, HttpServer, FixtureBackend): pybind11 shares registered types
// between the two modules, and both are built from the same sources by _build.py.
// `_native` must be imported first (the module does it).
#include <sched.h>
#include <sys/resource.h>

#include <chrono>
#include <thread>

#include <pybind11/functional.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "backend.h"
#include "fixture_backend.h"
#include "grpc_h2.h"
#include "httpd.h"
#include "loadgen.h"
#include "telemetry.h"

namespace py = pybind11;
using namespace amdgpu_dp;

PYBIND11_MODULE(_native_bench, m) {
  m.doc() = "Load generators and latency probes for the MI355X device plugin's benchmarks and tests";
  py::module_::import("k8s_gpu_device_plugin_amd._native");  // registers the shared types
  // per-call latency loops on a compiled client (methods of _native.H2Client)
  py::class_<H2Client> h2 = py::reinterpret_borrow<py::class_<H2Client>>(py::type::of<H2Client>());
  h2.def("bench_unary",
           [](H2Client& c, const std::string& path, const py::bytes& req, int n, int gap_us) {
             std::string r(req), resp, msg;
             std::vector<double> out;
             out.reserve(static_cast<size_t>(n));
             py::gil_scoped_release rel;
             for (int i = 0; i < n; ++i) {
               // gap_us > 0: idle between calls, so each one meets a sleeping server (the
               // way kubelet's sparse pod-admission RPCs do), not its busy-poll window
               if (gap_us > 0) std::this_thread::sleep_for(std::chrono::microseconds(gap_us));
               const int64_t t0 = mono_ns();
               const int st = c.unary(path, r, &resp, &msg);
               out.push_back((mono_ns() - t0) * 1e-9);
               if (st != 0) throw std::runtime_error("grpc-status " + std::to_string(st) + ": " + msg);
             }
             return out;
           },
           py::arg("path"), py::arg("req"), py::arg("n"), py::arg("gap_us") = 0);
  h2.def("bench_unary_ts",
         // Same as bench_unary, per call: (start, CLOCK_MONOTONIC ns; latency, s; the CPU the
         // client ran on when the answer arrived; involuntary context switches of the client
         // thread during the call, read outside the timed interval; ns from the last recv()
         // returning to the call's end, the client's own parsing) - for attributing the
         // tail to idle gaps, CPU migrations, preemption or the server's handling (the
         // server's own per-call record: grpc.callTraceFile).
         [](H2Client& c, const std::string& path, const py::bytes& req, int n, int gap_us) {
           std::string r(req), resp, msg;
           std::vector<int64_t> starts, tail_ns;
           std::vector<double> lat;
           std::vector<int> cpus, preempted;
           c.set_stamp_recv(true);
           starts.reserve(static_cast<size_t>(n));
           lat.reserve(static_cast<size_t>(n));
           cpus.reserve(static_cast<size_t>(n));
           preempted.reserve(static_cast<size_t>(n));
           {
             py::gil_scoped_release rel;
             struct rusage ru {};
             getrusage(RUSAGE_THREAD, &ru);
             long ivcsw = ru.ru_nivcsw;
             for (int i = 0; i < n; ++i) {
               if (gap_us > 0) std::this_thread::sleep_for(std::chrono::microseconds(gap_us));
               const int64_t t0 = mono_ns();
               const int st = c.unary(path, r, &resp, &msg);
               const int64_t t1 = mono_ns();
               lat.push_back((t1 - t0) * 1e-9);
               starts.push_back(t0);
               tail_ns.push_back(t1 - c.last_recv_ns());  // after the last recv returned
               cpus.push_back(sched_getcpu());
               getrusage(RUSAGE_THREAD, &ru);
               preempted.push_back(static_cast<int>(ru.ru_nivcsw - ivcsw));
               ivcsw = ru.ru_nivcsw;
               if (st != 0) throw std::runtime_error("grpc-status " + std::to_string(st) + ": " + msg);
             }
           }
           c.set_stamp_recv(false);
           return py::make_tuple(starts, lat, cpus, preempted, tail_ns);
         },
         py::arg("path"), py::arg("req"), py::arg("n"), py::arg("gap_us") = 0);

  m.def("h2_bench_unary",
        [](const std::string& sock, const std::string& path, const py::bytes& req, int n) {
          std::string r(req);
          py::gil_scoped_release rel;
          return h2_bench_unary(sock, path, r, n);
        });

  // ---- load generators (bench / BASELINE protocol) ----
  auto load_dict = [](const LoadResult& r) {
    py::dict d;
    d["ok"] = r.ok;
    d["errors"] = r.errors;
    d["bytes"] = r.bytes;
    d["elapsed_s"] = r.elapsed_s;
    d["latencies_s"] = r.latencies_s;
    return d;
  };
  m.def("http_load",
        [load_dict](const std::string& host, int port, const std::string& path, int conns, double duration_s,
                    double target_rps, bool accept_gzip) {
          LoadResult r;
          {
            py::gil_scoped_release rel;
            r = http_load(host, port, path, conns, duration_s, target_rps, accept_gzip);
          }
          return load_dict(r);
        },
        py::arg("host"), py::arg("port"), py::arg("path") = "/metrics", py::arg("conns") = 4,
        py::arg("duration_s") = 2.0, py::arg("target_rps") = 0.0, py::arg("accept_gzip") = false);
  m.def(
      "health_propagation",
      [](std::shared_ptr<Backend> be, const std::string& sock, int gpu, int events) {
        auto* fx = dynamic_cast<FixtureBackend*>(be.get());
        if (!fx) throw std::invalid_argument("health_propagation needs a fixture backend");
        py::gil_scoped_release rel;
        return health_propagation(*fx, sock, gpu, events);
      },
      py::arg("backend"), py::arg("socket_path"), py::arg("gpu"), py::arg("events") = 60);
  m.def("uds_pingpong",
        [](int n, int warmup, int req_bytes, int resp_bytes, bool server_spin, bool tcp, int gap_us, int client_cpu,
           int server_cpu, bool peek) {
          py::gil_scoped_release rel;
          return uds_pingpong(n, warmup, req_bytes, resp_bytes, server_spin, tcp, gap_us, client_cpu, server_cpu, peek);
        },
        py::arg("n") = 10000, py::arg("warmup") = 500, py::arg("req_bytes") = 128, py::arg("resp_bytes") = 256,
        py::arg("server_spin") = false, py::arg("tcp") = false, py::arg("gap_us") = 0, py::arg("client_cpu") = -1,
        py::arg("server_cpu") = -1, py::arg("peek") = false);
  m.def("core_ghz",
        [](int64_t iters, int reps) {
          py::gil_scoped_release rel;
          return core_ghz(iters, reps);
        },
        py::arg("iters") = 20000000, py::arg("reps") = 5);
  m.def("uds_pingpong_batched",
        [](int batches, int batch, int batch_gap_us, int req_bytes, int resp_bytes, int server_poll_us) {
          py::gil_scoped_release rel;
          return uds_pingpong_batched(batches, batch, batch_gap_us, req_bytes, resp_bytes, server_poll_us);
        },
        py::arg("batches"), py::arg("batch"), py::arg("batch_gap_us"), py::arg("req_bytes"), py::arg("resp_bytes"),
        py::arg("server_poll_us") = 50);
  py::class_<UdsPinger>(m, "UdsPinger")
      .def(py::init<int, int, int>(), py::arg("req_bytes"), py::arg("resp_bytes"), py::arg("server_timeout_ms") = 100)
      .def("once", &UdsPinger::once, py::call_guard<py::gil_scoped_release>());
  m.def("render_bench",
        [](std::shared_ptr<Exporter> ex, std::shared_ptr<HttpServer> http, int threads, int iters) {
          py::gil_scoped_release rel;
          return render_bench(std::move(ex), std::move(http), threads, iters);
        },
        py::arg("exporter"), py::arg("http") = nullptr, py::arg("threads") = 1, py::arg("iters") = 10000);
  m.def("grpc_load",
        [load_dict](const std::string& sock, const std::string& method, const py::bytes& req, int conns,
                    double duration_s) {
          std::string rq(req);
          LoadResult r;
          {
            py::gil_scoped_release rel;
            r = grpc_load(sock, method, rq, conns, duration_s);
          }
          return load_dict(r);
        },
        py::arg("socket_path"), py::arg("method"), py::arg("req"), py::arg("conns") = 4, py::arg("duration_s") = 2.0);
}
