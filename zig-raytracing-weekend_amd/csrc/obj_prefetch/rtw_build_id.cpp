extern "C" const char* rtw_build_id(void) { return "656b68882655f844"; }
