# jpge build (no cmake needed).  `make -j8` builds:
#   jpgenc_amd/lib/libjpge.so   the product: HIP kernels for gfx950 + host C++ + C ABI
#   jpgenc_amd/bin/jpgenc       the CLI (reference main.cpp contract)
#   oracle/build/liborc.so      test-only CPU restatement (+ oracle/_ref when /root/reference exists)
ROCM     ?= /opt/rocm
HIPCC    ?= $(ROCM)/bin/hipcc
CXX      ?= g++
ARCH     ?= gfx950
BUILD    ?= build/obj
SRC      := jpgenc_amd/csrc
LIBDIR   ?= jpgenc_amd/lib
BINDIR   := jpgenc_amd/bin

HIPFLAGS := --offload-arch=$(ARCH) -O3 -std=c++17 -fPIC -ffp-contract=off -I$(SRC) -Iinclude $(HIPEXTRA)
CXXFLAGS := -O2 -std=c++17 -fPIC -pthread -Wall -Wextra -Wno-unused-parameter -Wno-unused-result \
            -D__HIP_PLATFORM_AMD__ -I$(ROCM)/include -I$(SRC) -Iinclude $(HIPEXTRA)

HOST_SRCS := encoder.cpp capi.cpp host_io.cpp huffman.cpp jpge_image.cpp ingest.cpp host_decode.cpp coding.cpp group.cpp
HOST_OBJS := $(addprefix $(BUILD)/,$(HOST_SRCS:.cpp=.o))
DEV_SRCS  := fdct.hip stats.hip entropy.hip planes.hip concat.hip
DEV_OBJS  := $(addprefix $(BUILD)/,$(DEV_SRCS:.hip=.o))
DIAG_OBJS := $(addprefix $(BUILD)/diag/,$(DEV_SRCS:.hip=.o))
HEADERS   := $(wildcard $(SRC)/*.hpp) include/jpge.h
FACADE_TEST := tests/cpp/bin/test_facade
HUFF_TEST   := tests/cpp/bin/test_huffman_fast
QUANT_TEST  := tests/cpp/bin/test_quant_fast
EXIT_TEST   := tests/cpp/bin/test_exit_close

all: $(LIBDIR)/libjpge.so $(BINDIR)/jpgenc $(FACADE_TEST) $(HUFF_TEST) $(QUANT_TEST) $(EXIT_TEST) oracle

$(BUILD)/%.o: $(SRC)/%.hip $(HEADERS)
	@mkdir -p $(BUILD)
	$(HIPCC) $(HIPFLAGS) -c $< -o $@

$(BUILD)/diag/%.o: $(SRC)/%.hip $(HEADERS)
	@mkdir -p $(BUILD)/diag
	$(HIPCC) $(HIPFLAGS) -DJPGE_STAMPS -c $< -o $@

$(BUILD)/%.o: $(SRC)/%.cpp $(HEADERS)
	@mkdir -p $(BUILD)
	$(CXX) $(CXXFLAGS) -c $< -o $@

$(LIBDIR)/libjpge.so: $(DEV_OBJS) $(HOST_OBJS)
	@mkdir -p $(LIBDIR)
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -pthread -o $@ $^ -L$(ROCM)/lib -lamdhip64 -ldl

$(BINDIR)/jpgenc: $(SRC)/cli.cpp $(LIBDIR)/libjpge.so
	@mkdir -p $(BINDIR)
	$(CXX) $(CXXFLAGS) -o $@ $< -L$(LIBDIR) -ljpge -Wl,-rpath,'$$ORIGIN/../lib' \
	  -L$(ROCM)/lib -lamdhip64 -Wl,-rpath,$(ROCM)/lib

oracle:
	$(MAKE) -C oracle

# diagnostic build with in-kernel phase stamps (JPGE_LIB=jpgenc_amd/lib/diag/libjpge.so,
# JPGE_STAMPS_FILE=<path>); never used by tests or the bench
diag: $(DIAG_OBJS) $(HOST_OBJS)
	@mkdir -p $(LIBDIR)/diag
	$(HIPCC) --offload-arch=$(ARCH) -shared -fPIC -pthread -o $(LIBDIR)/diag/libjpge.so $^ \
	  -L$(ROCM)/lib -lamdhip64

clean:
	rm -rf build $(LIBDIR) $(BINDIR) tests/cpp/bin
	$(MAKE) -C oracle clean

.PHONY: all oracle clean

# the facade under the reference's unit tests (tests/cpp/test_facade.cpp; run by
# tests/test_facade.py): compiled exactly as reference code would be, global names
$(FACADE_TEST): tests/cpp/test_facade.cpp $(LIBDIR)/libjpge.so $(SRC)/jpge_image.hpp include/jpge.h
	@mkdir -p tests/cpp/bin
	$(CXX) $(CXXFLAGS) -o $@ $< -L$(LIBDIR) -ljpge -Wl,-rpath,'$$ORIGIN/../../../$(LIBDIR)' \
	  -L$(ROCM)/lib -lamdhip64 -Wl,-rpath,$(ROCM)/lib

# a caller's exit-time close after the library's own exit handler (tests/test_gpu_teardown.py)
$(EXIT_TEST): tests/cpp/test_exit_close.cpp $(LIBDIR)/libjpge.so include/jpge.h
	@mkdir -p tests/cpp/bin
	$(CXX) $(CXXFLAGS) -o $@ $< -L$(LIBDIR) -ljpge -Wl,-rpath,'$$ORIGIN/../../../$(LIBDIR)' \
	  -L$(ROCM)/lib -lamdhip64 -Wl,-rpath,$(ROCM)/lib

# the Huffman table builder's array emulation against the standard containers
# (tests/test_host.py runs it)
$(HUFF_TEST): tests/cpp/test_huffman_fast.cpp $(SRC)/huffman.cpp $(SRC)/huffman.hpp
	@mkdir -p tests/cpp/bin
	$(CXX) $(CXXFLAGS) -o $@ $< $(SRC)/huffman.cpp

# K1's quantiser fast path against the reference's two roundings (tests/test_host.py runs it)
$(QUANT_TEST): tests/cpp/test_quant_fast.cpp $(SRC)/constants.hpp
	@mkdir -p tests/cpp/bin
	$(CXX) -O2 -std=c++17 -ffp-contract=off -I$(SRC) -o $@ $<

# Host code under AddressSanitizer + UndefinedBehaviorSanitizer (run by
# tests/test_asan.py in the CPU suite): every host .cpp of the library rebuilt
# sanitized and linked with the (unsanitized) HIP device objects, plus the host
# tests.  No GPU is touched: the drivers call host-only entry points.
ASAN_FLAGS := -fsanitize=address,undefined -fno-sanitize-recover=all -fno-omit-frame-pointer -g -O1
ASAN_DIR   := build/asan
ASAN_BIN   := tests/cpp/bin/asan
ASAN_OBJS  := $(addprefix $(ASAN_DIR)/,$(HOST_SRCS:.cpp=.o))
ASAN_TESTS := $(ASAN_BIN)/test_host_asan $(ASAN_BIN)/test_facade $(ASAN_BIN)/test_huffman_fast $(ASAN_BIN)/test_quant_fast

$(ASAN_DIR)/%.o: $(SRC)/%.cpp $(HEADERS)
	@mkdir -p $(ASAN_DIR)
	$(CXX) $(CXXFLAGS) $(ASAN_FLAGS) -c $< -o $@

$(ASAN_BIN)/test_host_asan: tests/cpp/test_host_asan.cpp $(ASAN_OBJS) $(DEV_OBJS)
	@mkdir -p $(ASAN_BIN)
	$(CXX) $(CXXFLAGS) $(ASAN_FLAGS) -o $@ $^ -L$(ROCM)/lib -lamdhip64 -ldl -Wl,-rpath,$(ROCM)/lib

$(ASAN_BIN)/test_facade: tests/cpp/test_facade.cpp $(ASAN_OBJS) $(DEV_OBJS)
	@mkdir -p $(ASAN_BIN)
	$(CXX) $(CXXFLAGS) $(ASAN_FLAGS) -o $@ $^ -L$(ROCM)/lib -lamdhip64 -ldl -Wl,-rpath,$(ROCM)/lib

$(ASAN_BIN)/test_huffman_fast: tests/cpp/test_huffman_fast.cpp $(SRC)/huffman.cpp $(SRC)/huffman.hpp
	@mkdir -p $(ASAN_BIN)
	$(CXX) $(CXXFLAGS) $(ASAN_FLAGS) -o $@ $< $(SRC)/huffman.cpp

$(ASAN_BIN)/test_quant_fast: tests/cpp/test_quant_fast.cpp $(SRC)/constants.hpp
	@mkdir -p $(ASAN_BIN)
	$(CXX) -std=c++17 -ffp-contract=off -I$(SRC) $(ASAN_FLAGS) -o $@ $<

asan: $(ASAN_TESTS)

.PHONY: asan
