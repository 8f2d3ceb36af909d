// pybind11 bindings of the CPU runtime library (_vwa_native): grammar engine + mask cache.
#include <pybind11/numpy.h>
#include <pybind11/pybind11.h>
#include <pybind11/stl.h>

#include "grammar.h"
#include "shm_channel.h"

namespace py = pybind11;
using namespace vwa;

PYBIND11_MODULE(_vwa_native, m) {
  m.doc() = "voice-web-agent native runtime: JSON-schema constrained decoding";
  py::class_<Grammar, std::shared_ptr<Grammar>>(m, "Grammar")
      .def(py::init<const std::string&>())
      .def("n_nodes", &Grammar::n_nodes)
      .def("root", &Grammar::root);
  py::class_<Vocab, std::shared_ptr<Vocab>>(m, "Vocab")
      .def(py::init([](const std::vector<py::bytes>& toks, const std::vector<int>& eos) {
        std::vector<std::string> t;
        t.reserve(toks.size());
        for (auto& b : toks) t.emplace_back(std::string(b));
        return std::make_shared<Vocab>(t, eos);
      }))
      .def("size", &Vocab::size)
      .def("words", &Vocab::words)
      .def("max_len", &Vocab::max_len)
      .def("n_special_trie_nodes", [](const Vocab& v) { return v.spec_nodes.size(); })
      .def("n_full_trie_nodes", [](const Vocab& v) { return v.full_nodes.size(); });
  py::class_<Compiled, std::shared_ptr<Compiled>>(m, "Compiled")
      .def(py::init<std::shared_ptr<Grammar>, std::shared_ptr<Vocab>, size_t>(), py::arg("grammar"), py::arg("vocab"),
           py::arg("cache_cap") = 4096)
      .def_readonly("hits", &Compiled::hits)
      .def_readonly("misses", &Compiled::misses)
      .def_readonly("miss_ms", &Compiled::miss_ms);
  py::class_<Matcher>(m, "Matcher")
      .def(py::init<std::shared_ptr<Compiled>, int>(), py::arg("compiled"), py::arg("budget") = 1 << 30)
      .def("accept_bytes", [](Matcher& mt, py::bytes b) { return mt.accept_bytes(std::string(b)); })
      .def("accept_token", &Matcher::accept_token)
      .def("can_accept_token", &Matcher::can_accept_token)
      .def("fill_mask",
           [](const Matcher& mt, py::array_t<int32_t, py::array::c_style> out) {
             auto buf = out.mutable_unchecked<1>();
             if ((int)buf.shape(0) < mt.compiled()->v->words()) throw std::runtime_error("mask buffer too small");
             py::gil_scoped_release rel;
             mt.fill_mask(reinterpret_cast<uint32_t*>(out.mutable_data()));
           })
      .def("forced_prefix", [](const Matcher& mt, int max_len) { return py::bytes(mt.forced_prefix(max_len)); },
           py::arg("max_len") = 256)
      .def("is_accept", &Matcher::is_accept)
      .def("used", &Matcher::used)
      .def("budget", &Matcher::budget)
      .def("min_completion", &Matcher::min_completion)
      .def("canon", [](const Matcher& mt) { return py::bytes(mt.canon()); })
      .def("clone", &Matcher::clone);
  // TP brain control plane (brain/tp_engine.py): /dev/shm broadcast ring, waits without the GIL
  py::class_<ShmChannel>(m, "ShmChannel")
      .def(py::init<const std::string&, int, int64_t, int, bool>(), py::arg("name"), py::arg("n_readers") = 1,
           py::arg("slot_bytes") = 1 << 20, py::arg("n_slots") = 4, py::arg("create") = false)
      .def("publish",
           [](ShmChannel& c, py::bytes b, double timeout_s) {
             std::string s(b);
             py::gil_scoped_release rel;
             return c.publish(s, timeout_s);
           },
           py::arg("payload"), py::arg("timeout_s") = 60.0)
      .def("receive",
           [](ShmChannel& c, int r, double timeout_s, double dead_s) {
             std::string s;
             {
               py::gil_scoped_release rel;
               s = c.receive(r, timeout_s, dead_s);
             }
             return py::bytes(s);
           },
           py::arg("reader"), py::arg("timeout_s") = -1.0, py::arg("dead_s") = 60.0)
      .def("beat", &ShmChannel::beat)
      .def("unlink", &ShmChannel::unlink)
      .def("published", &ShmChannel::published)
      .def("acked", &ShmChannel::acked)
      .def_property_readonly("n_readers", &ShmChannel::n_readers)
      .def_property_readonly("slot_bytes", &ShmChannel::slot_bytes);
}
