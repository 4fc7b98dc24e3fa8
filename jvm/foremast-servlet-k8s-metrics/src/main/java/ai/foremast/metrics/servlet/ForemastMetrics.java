package ai.foremast.metrics.servlet;

import io.micrometer.core.instrument.Tag;
import io.micrometer.core.instrument.Timer;
import io.micrometer.core.instrument.binder.jvm.JvmGcMetrics;
import io.micrometer.core.instrument.binder.jvm.JvmMemoryMetrics;
import io.micrometer.core.instrument.binder.jvm.JvmThreadMetrics;
import io.micrometer.core.instrument.binder.system.ProcessorMetrics;
import io.micrometer.prometheus.PrometheusConfig;
import io.micrometer.prometheus.PrometheusMeterRegistry;

import java.time.Duration;
import java.util.ArrayList;
import java.util.List;
import java.util.Map;

/**
 * One registry per application with the series the foremast recording rules
 * read (deploy/foremast/22-recording-rules.yaml), for services outside Spring
 * Boot 2 (Spring 4 MVC, Boot 1.x, plain servlet containers):
 * <ul>
 *   <li>common tags -- {@code app} from {@code APP_NAME} (env) or the
 *       {@code app} init parameter -- on every meter;</li>
 *   <li>{@code http.server.requests} timers with 0.95 / 0.98 percentiles,
 *       recorded by {@link HttpRequestsFilter};</li>
 *   <li>zero-valued timers for the statuses of {@code initializeForStatuses}
 *       (403, 404, 500, 503 by default), so an error-rate rule sees 0, not no
 *       series;</li>
 *   <li>JVM memory / GC / thread and CPU binders (the rules' jvm_* and cpu
 *       series); Tomcat session meters through {@link ForemastMetricsListener};</li>
 *   <li>the common-metrics gate ({@link CommonMetricsGate}: whitelist,
 *       blacklist, prefixes, tag rules, runtime enable / disable through
 *       {@link MetricsControlServlet}).</li>
 * </ul>
 * {@link PrometheusScrapeServlet} exposes it.  Same names and tags as the Boot 2
 * starter and foremast_amd/emitter/metrics.py.
 */
public final class ForemastMetrics {

    public static final String HTTP_REQUESTS = "http.server.requests";

    private static volatile ForemastMetrics shared;

    private final PrometheusMeterRegistry registry;
    private final String callerHeader;
    private final String callerDefault;
    private final CommonMetricsGate gate;

    public ForemastMetrics(Map<String, String> settings) {
        this.registry = new PrometheusMeterRegistry(PrometheusConfig.DEFAULT);
        // the common-metrics gate sees every meter: registered before any
        this.gate = new CommonMetricsGate(settings);
        registry.config().meterFilter(gate);
        List<Tag> common = new ArrayList<>();
        String app = first(System.getenv("APP_NAME"), settings.get("app"));
        if (app != null) {
            common.add(Tag.of("app", app));
        }
        registry.config().commonTags(common);
        this.callerHeader = first(settings.get("callerHeader"), "X-CALLER");
        // a request without the caller header: the reference's "UNKNOWN"
        // (CallerWebMvcTagsProvider.java:14), configurable
        this.callerDefault = first(settings.get("callerDefault"), "UNKNOWN");
        registry.config().meterFilter(new io.micrometer.core.instrument.config.MeterFilter() {
            @Override
            public io.micrometer.core.instrument.distribution.DistributionStatisticConfig configure(
                    io.micrometer.core.instrument.Meter.Id id,
                    io.micrometer.core.instrument.distribution.DistributionStatisticConfig config) {
                if (!HTTP_REQUESTS.equals(id.getName()) || config.getPercentiles() != null) {
                    return config;
                }
                return io.micrometer.core.instrument.distribution.DistributionStatisticConfig.builder()
                        .percentiles(0.95, 0.98).expiry(Duration.ofMinutes(2)).build().merge(config);
            }
        });
        String statuses = first(settings.get("initializeForStatuses"), "403,404,500,503");
        for (String s : statuses.split(",")) {
            String status = s.trim();
            if (!status.isEmpty()) {
                Timer.builder(HTTP_REQUESTS).tags("exception", "None", "method", "GET", "outcome",
                        HttpRequestsFilter.outcome(Integer.parseInt(status)), "status", status, "uri", "/**",
                        "caller", "*").register(registry);
            }
        }
        if (!"false".equals(settings.get("jvmMetrics"))) {
            new JvmMemoryMetrics().bindTo(registry);
            new JvmGcMetrics().bindTo(registry);
            new JvmThreadMetrics().bindTo(registry);
            new ProcessorMetrics().bindTo(registry);
        }
    }

    /** The application-wide instance (created by the first filter / servlet that asks). */
    public static ForemastMetrics shared(Map<String, String> settings) {
        ForemastMetrics m = shared;
        if (m == null) {
            synchronized (ForemastMetrics.class) {
                if (shared == null) {
                    shared = new ForemastMetrics(settings);
                }
                m = shared;
            }
        }
        return m;
    }

    public PrometheusMeterRegistry registry() {
        return registry;
    }

    public String callerHeader() {
        return callerHeader;
    }

    public String callerDefault() {
        return callerDefault;
    }

    public CommonMetricsGate gate() {
        return gate;
    }

    static String first(String a, String b) {
        return a != null && !a.trim().isEmpty() ? a.trim() : (b != null && !b.trim().isEmpty() ? b.trim() : null);
    }
}
