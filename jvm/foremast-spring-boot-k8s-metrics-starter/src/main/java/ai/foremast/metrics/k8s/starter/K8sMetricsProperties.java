package ai.foremast.metrics.k8s.starter;

import org.springframework.boot.context.properties.ConfigurationProperties;

/**
 * {@code k8s.metrics.*}: the knobs of the foremast in-app metrics.  Names and
 * defaults match {@code foremast_amd/emitter/metrics.py:K8sMetricsProperties},
 * so a Python and a JVM service of one fleet are configured alike.
 */
@ConfigurationProperties(prefix = "k8s.metrics")
public class K8sMetricsProperties {

    /** {@code tag:SOURCE|SOURCE,...}; a source is {@code ENV.VAR}, an application property or a literal. */
    private String commonTagNameValuePairs = "app:ENV.APP_NAME|info.app.name";

    /** HTTP statuses whose request timers exist (at zero) before the first such response. */
    private String initializeForStatuses = "403,404,500,503";

    /** Header carrying the calling service; its value becomes the {@code caller} tag (empty: no tag). */
    private String callerHeader = "X-CALLER";

    /** The caller tag of a request without the caller header (the reference's "UNKNOWN"). */
    private String callerDefault = "UNKNOWN";

    /** Hide every meter that is not enabled explicitly, whitelisted, prefixed or tag-matched. */
    private boolean enableCommonMetricsFilter = false;

    /** Allow {@code POST /actuator/k8s-metrics/{enable|disable}/{metric}} at runtime. */
    private boolean enableCommonMetricsFilterAction = false;

    private String commonMetricsWhitelist;
    private String commonMetricsBlacklist;
    private String commonMetricsPrefix;
    /** {@code tag:value,...}: a meter carrying any of these tag values is exposed. */
    private String commonMetricsTagRules;

    /** Serve {@code /metrics} as the Prometheus scrape (what Kubernetes scrapes by default). */
    private boolean metricsPathAlias = true;

    /** Disable CSRF for the actuator endpoints (POST enable/disable from kubectl plugins). */
    private boolean disableCsrf = false;

    public String getCommonTagNameValuePairs() { return commonTagNameValuePairs; }
    public void setCommonTagNameValuePairs(String v) { commonTagNameValuePairs = v; }
    public String getInitializeForStatuses() { return initializeForStatuses; }
    public void setInitializeForStatuses(String v) { initializeForStatuses = v; }
    public String getCallerHeader() { return callerHeader; }
    public void setCallerHeader(String v) { callerHeader = v; }
    public String getCallerDefault() { return callerDefault; }
    public void setCallerDefault(String v) { callerDefault = v; }
    public boolean isEnableCommonMetricsFilter() { return enableCommonMetricsFilter; }
    public void setEnableCommonMetricsFilter(boolean v) { enableCommonMetricsFilter = v; }
    public boolean isEnableCommonMetricsFilterAction() { return enableCommonMetricsFilterAction; }
    public void setEnableCommonMetricsFilterAction(boolean v) { enableCommonMetricsFilterAction = v; }
    public String getCommonMetricsWhitelist() { return commonMetricsWhitelist; }
    public void setCommonMetricsWhitelist(String v) { commonMetricsWhitelist = v; }
    public String getCommonMetricsBlacklist() { return commonMetricsBlacklist; }
    public void setCommonMetricsBlacklist(String v) { commonMetricsBlacklist = v; }
    public String getCommonMetricsPrefix() { return commonMetricsPrefix; }
    public void setCommonMetricsPrefix(String v) { commonMetricsPrefix = v; }
    public String getCommonMetricsTagRules() { return commonMetricsTagRules; }
    public void setCommonMetricsTagRules(String v) { commonMetricsTagRules = v; }
    public boolean isMetricsPathAlias() { return metricsPathAlias; }
    public void setMetricsPathAlias(boolean v) { metricsPathAlias = v; }
    public boolean isDisableCsrf() { return disableCsrf; }
    public void setDisableCsrf(boolean v) { disableCsrf = v; }
}
