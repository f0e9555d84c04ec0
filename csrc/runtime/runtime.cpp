// pybind11 bindings of the control-plane runtime core (runtime_core.h) as
// `kubeflow_controller_amd._native_runtime`.  Everything blocking releases the GIL.
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "runtime_core.h"

namespace py = pybind11;

// ----------------------------------------------------------------------------- module
PYBIND11_MODULE(_native_runtime, m) {
  m.doc() = "Native control-plane runtime: workqueue, rate limiters, expectations, process launcher";
  m.def("set_fake_clock", [](double t) { g_fake_now = t; g_fake = true; });
  m.def("advance_fake_clock", [](double dt) { g_fake_now = g_fake_now.load() + dt; });
  m.def("use_real_clock", [] { g_fake = false; });
  m.def("now", &now_s);

  py::class_<RateLimiter, std::shared_ptr<RateLimiter>>(m, "RateLimiter")
      .def("when", &RateLimiter::when)
      .def("forget", &RateLimiter::forget)
      .def("num_requeues", &RateLimiter::num_requeues);
  py::class_<ExpFailureLimiter, RateLimiter, std::shared_ptr<ExpFailureLimiter>>(m, "ItemExponentialFailureRateLimiter")
      .def(py::init<double, double>(), py::arg("base_delay") = 0.005, py::arg("max_delay") = 1000.0);
  py::class_<BucketLimiter, RateLimiter, std::shared_ptr<BucketLimiter>>(m, "BucketRateLimiter")
      .def(py::init<double, int>(), py::arg("qps") = 10.0, py::arg("burst") = 100);
  py::class_<MaxOfLimiter, RateLimiter, std::shared_ptr<MaxOfLimiter>>(m, "MaxOfRateLimiter")
      .def(py::init<std::vector<std::shared_ptr<RateLimiter>>>());
  m.def("default_controller_rate_limiter", &default_controller_rate_limiter);

  py::class_<WorkQueue>(m, "RateLimitingQueue")
      .def(py::init([](std::shared_ptr<RateLimiter> l, std::string name) {
             return new WorkQueue(std::move(name), l ? l : default_controller_rate_limiter());
           }),
           py::arg("rate_limiter") = nullptr, py::arg("name") = "")
      .def("add", &WorkQueue::add)
      .def("__len__", &WorkQueue::len)
      .def("get",
           [](WorkQueue &q, double timeout) {
             std::pair<std::optional<std::string>, bool> r;
             {
               py::gil_scoped_release nogil;
               r = q.get(timeout);
             }
             return py::make_tuple(r.first ? py::object(py::str(*r.first)) : py::object(py::none()), r.second);
           },
           py::arg("timeout") = -1.0)
      .def("done", &WorkQueue::done)
      .def("shut_down", &WorkQueue::shut_down)
      .def("shutting_down", &WorkQueue::shutting_down)
      .def("add_after", &WorkQueue::add_after)
      .def("add_rate_limited", &WorkQueue::add_rate_limited)
      .def("forget", &WorkQueue::forget)
      .def("num_requeues", &WorkQueue::num_requeues)
      .def("num_waiting", &WorkQueue::num_waiting)
      .def("poll_delayed", &WorkQueue::poll_delayed)
      .def_property_readonly("name", &WorkQueue::name);

  py::class_<Expectations>(m, "ControllerExpectations")
      .def(py::init<double>(), py::arg("ttl") = 300.0)
      .def("satisfied_expectations", &Expectations::satisfied)
      .def("set_expectations", &Expectations::set)
      .def("expect_creations", [](Expectations &e, const std::string &k, long n) { e.set(k, n, 0); })
      .def("expect_deletions", [](Expectations &e, const std::string &k, long n) { e.set(k, 0, n); })
      .def("raise_expectations", &Expectations::raise)
      .def("lower_expectations", &Expectations::lower)
      .def("creation_observed", [](Expectations &e, const std::string &k) { e.lower(k, 1, 0); })
      .def("deletion_observed", [](Expectations &e, const std::string &k) { e.lower(k, 0, 1); })
      .def("delete_expectations", &Expectations::erase)
      .def("get_expectations", &Expectations::get);

  m.def("spawn", &spawn_process, py::arg("argv"), py::arg("env"), py::arg("cwd") = "", py::arg("log_path") = "");
  m.def("poll", &poll_process);
  m.def("kill_group", &kill_group);
  m.def("pid_alive", &pid_alive);
}
