# Builds the MI355X (gfx950) product library + CLI, the CPU oracle and the synthetic-data tool.
#   make            -> pwasm_amd/lib/libpwasm_amd.so, pwasm_amd/bin/pafreport,
#                      oracle/build/*, synth/build/pwsynth
HIPCC    ?= /opt/rocm/bin/hipcc
ARCH     ?= gfx950
HIPFLAGS ?= -O3 -std=c++17 -fPIC --offload-arch=$(ARCH) -Wall -Wno-unused-function
INC      := -Iinclude -Ipwasm_amd/csrc
SRC_DIR  := pwasm_amd/csrc
OBJ_DIR  := pwasm_amd/build
LIB      := pwasm_amd/lib/libpwasm_amd.so
CLI      := pwasm_amd/bin/pafreport
OBJS     := $(OBJ_DIR)/pw_report.o $(OBJ_DIR)/pw_host.o $(OBJ_DIR)/pw_msa.o $(OBJ_DIR)/pw_gapassem.o $(OBJ_DIR)/pw_msa_layout.o $(OBJ_DIR)/pw_ga_api.o $(OBJ_DIR)/pw_msa_comm.o $(OBJ_DIR)/pw_pack.o
GA_CLI   := pwasm_amd/bin/gapassem_consensus

all: $(LIB) $(CLI) $(GA_CLI) oracle synth

$(OBJ_DIR):
	mkdir -p $(OBJ_DIR) pwasm_amd/lib pwasm_amd/bin

$(OBJ_DIR)/%.o: $(SRC_DIR)/%.hip $(SRC_DIR)/pw_tables.h $(SRC_DIR)/pw_wave.h include/pwasm_amd.h | $(OBJ_DIR)
	$(HIPCC) $(HIPFLAGS) $(INC) -c $< -o $@

# the report kernels: the scheduler strategy that clusters memory instructions (same-call sweep:
# index 127 -> 122 us, the rest unchanged; tools/exp_build.py s_maxmem)
$(OBJ_DIR)/pw_report.o: $(SRC_DIR)/pw_report.hip $(SRC_DIR)/pw_tables.h $(SRC_DIR)/pw_wave.h include/pwasm_amd.h | $(OBJ_DIR)
	$(HIPCC) $(HIPFLAGS) -mllvm -amdgpu-sched-strategy=max-memory-clause $(INC) -c $< -o $@

$(OBJ_DIR)/%.o: $(SRC_DIR)/%.cpp $(SRC_DIR)/pw_tables.h include/pwasm_amd.h include/pwasm_gapassem.hpp $(SRC_DIR)/pw_msa_layout.h | $(OBJ_DIR)
	$(HIPCC) $(HIPFLAGS) $(INC) -c $< -o $@

$(LIB): $(OBJS)
	$(HIPCC) -shared -fPIC --offload-arch=$(ARCH) -o $@ $(OBJS) -ldl

$(CLI): $(SRC_DIR)/pafreport_main.cpp $(LIB)
	$(HIPCC) -O2 -std=c++17 $(INC) -o $@ $< -Lpwasm_amd/lib -lpwasm_amd -Wl,-rpath,'$$ORIGIN/../lib'

$(GA_CLI): $(SRC_DIR)/gapassem_main.cpp $(LIB)
	$(HIPCC) -O2 -std=c++17 $(INC) -o $@ $< -Lpwasm_amd/lib -lpwasm_amd -Wl,-rpath,'$$ORIGIN/../lib'

oracle:
	$(MAKE) -C oracle

synth:
	$(MAKE) -C synth

clean:
	rm -rf $(OBJ_DIR) pwasm_amd/lib pwasm_amd/bin
	$(MAKE) -C oracle clean
	$(MAKE) -C synth clean

.PHONY: all oracle synth clean
