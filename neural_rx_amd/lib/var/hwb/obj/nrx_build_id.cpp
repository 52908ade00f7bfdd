extern "C" const char* nrx_build_id(void) { return "fb63bf08e13a69f6+-DNRX_RR_HEADS_GLB=0"; }
