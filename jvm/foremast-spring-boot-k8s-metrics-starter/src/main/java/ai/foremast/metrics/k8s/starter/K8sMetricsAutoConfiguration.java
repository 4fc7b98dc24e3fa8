package ai.foremast.metrics.k8s.starter;

import io.micrometer.core.instrument.MeterRegistry;
import io.micrometer.core.instrument.Tag;
import io.micrometer.core.instrument.Timer;
import io.micrometer.core.instrument.config.MeterFilter;
import io.micrometer.core.instrument.distribution.DistributionStatisticConfig;
import io.micrometer.core.instrument.Meter;
import org.springframework.boot.actuate.autoconfigure.metrics.MeterRegistryCustomizer;
import org.springframework.boot.actuate.autoconfigure.metrics.MetricsProperties;
import org.springframework.boot.autoconfigure.AutoConfiguration;
import org.springframework.boot.autoconfigure.condition.ConditionalOnClass;
import org.springframework.boot.autoconfigure.condition.ConditionalOnMissingBean;
import org.springframework.boot.autoconfigure.condition.ConditionalOnProperty;
import org.springframework.boot.autoconfigure.condition.ConditionalOnWebApplication;
import org.springframework.boot.context.properties.EnableConfigurationProperties;
import org.springframework.boot.web.servlet.FilterRegistrationBean;
import org.springframework.context.annotation.Bean;
import org.springframework.context.annotation.Configuration;
import org.springframework.core.env.Environment;

import javax.servlet.Filter;
import javax.servlet.RequestDispatcher;
import javax.servlet.http.HttpServletRequest;
import java.time.Duration;
import java.util.ArrayList;
import java.util.List;

/**
 * Wires the foremast in-app metrics into a Spring Boot 2 service:
 * <ul>
 *   <li>common tags ({@code app} by default) on every meter, resolved from
 *       {@code k8s.metrics.common-tag-name-value-pairs};</li>
 *   <li>{@code http.server.requests} with the {@code caller} tag, 0.95 / 0.98
 *       percentiles and zero-valued timers for {@code initialize-for-statuses},
 *       so the recording rules in deploy/foremast/22-recording-rules.yaml see a
 *       0 error rate instead of no series;</li>
 *   <li>the common-metrics gate ({@link MeterGate}) and its runtime endpoint;</li>
 *   <li>{@code /metrics} answered by the Prometheus scrape.</li>
 * </ul>
 * The Python services of a fleet get the same from foremast_amd/emitter/metrics.py.
 */
@AutoConfiguration
@ConditionalOnClass(MeterRegistry.class)
@EnableConfigurationProperties(K8sMetricsProperties.class)
public class K8sMetricsAutoConfiguration {

    static final String HTTP_REQUESTS = "http.server.requests";

    /** {@code tag:SRC|SRC,...} to tags; the first source with a value wins. */
    static List<Tag> commonTags(String spec, Environment env) {
        List<Tag> tags = new ArrayList<>();
        for (String pair : MeterGate.tokens(spec)) {
            int colon = pair.indexOf(':');
            if (colon <= 0) {
                throw new IllegalArgumentException("Invalid common tag name value pair:" + pair);
            }
            String name = pair.substring(0, colon).trim();
            String value = null;
            for (String src : pair.substring(colon + 1).split("\\|")) {
                src = src.trim();
                if (src.startsWith("ENV.")) {
                    value = System.getenv(src.substring(4));
                } else if (env != null && env.containsProperty(src)) {
                    value = env.getProperty(src);
                } else if (!src.contains(".")) {
                    value = src;                      // a literal
                }
                if (value != null && !value.isEmpty()) {
                    break;
                }
            }
            if (value != null && !value.isEmpty()) {
                tags.add(Tag.of(name, value));
            }
        }
        return tags;
    }

    @Bean
    public MeterRegistryCustomizer<MeterRegistry> foremastCommonTags(K8sMetricsProperties props, Environment env) {
        List<Tag> tags = commonTags(props.getCommonTagNameValuePairs(), env);
        return registry -> registry.config().commonTags(tags);
    }

    @Bean
    public MeterFilter foremastRequestPercentiles() {
        return new MeterFilter() {
            @Override
            public DistributionStatisticConfig configure(Meter.Id id, DistributionStatisticConfig config) {
                if (!HTTP_REQUESTS.equals(id.getName()) || config.getPercentiles() != null) {
                    return config;
                }
                return DistributionStatisticConfig.builder().percentiles(0.95, 0.98)
                        .expiry(Duration.ofMinutes(2)).build().merge(config);
            }
        };
    }

    @Bean
    @ConditionalOnMissingBean
    public MeterGate foremastMeterGate(K8sMetricsProperties props, MetricsProperties metrics) {
        return new MeterGate(props, metrics.getEnable());
    }

    @Bean
    public MeterRegistryCustomizer<MeterRegistry> foremastGateAndZeroStatuses(K8sMetricsProperties props,
                                                                           MeterGate gate) {
        return registry -> {
            registry.config().meterFilter(gate);
            // exception=None, method=GET, uri=/**, caller=* per status: the same
            // series the Python emitter pre-creates
            for (String status : MeterGate.tokens(props.getInitializeForStatuses())) {
                Timer.builder(HTTP_REQUESTS)
                        .tags("exception", "None", "method", "GET", "outcome", outcome(status),
                              "status", status, "uri", "/**", "caller", "*")
                        .register(registry);
            }
        };
    }

    static String outcome(String status) {
        char c = status.isEmpty() ? '0' : status.charAt(0);
        switch (c) {
            case '1': return "INFORMATIONAL";
            case '2': return "SUCCESS";
            case '3': return "REDIRECTION";
            case '4': return "CLIENT_ERROR";
            case '5': return "SERVER_ERROR";
            default: return "UNKNOWN";
        }
    }

    @Bean
    @ConditionalOnMissingBean
    public K8sMetricsEndpoint foremastK8sMetricsEndpoint(MeterGate gate) {
        return new K8sMetricsEndpoint(gate);
    }

    @Configuration(proxyBeanMethods = false)
    @ConditionalOnWebApplication(type = ConditionalOnWebApplication.Type.SERVLET)
    @ConditionalOnClass(name = "org.springframework.boot.actuate.metrics.web.servlet.DefaultWebMvcTagsProvider")
    static class ServletMetrics {

        @Bean
        @ConditionalOnMissingBean(org.springframework.boot.actuate.metrics.web.servlet.WebMvcTagsProvider.class)
        public CallerTagsProvider foremastCallerTags(K8sMetricsProperties props) {
            return new CallerTagsProvider(props.getCallerHeader(), props.getCallerDefault());
        }

        /** {@code GET /metrics} forwarded to the actuator's Prometheus scrape. */
        @Bean
        @ConditionalOnProperty(prefix = "k8s.metrics", name = "metrics-path-alias", matchIfMissing = true)
        public FilterRegistrationBean<Filter> foremastMetricsAlias() {
            Filter alias = (req, res, chain) -> {
                HttpServletRequest http = (HttpServletRequest) req;
                if ("/metrics".equals(http.getRequestURI())) {
                    RequestDispatcher d = http.getRequestDispatcher("/actuator/prometheus");
                    d.forward(req, res);
                    return;
                }
                chain.doFilter(req, res);
            };
            FilterRegistrationBean<Filter> reg = new FilterRegistrationBean<>(alias);
            reg.addUrlPatterns("/metrics");
            reg.setOrder(0);
            return reg;
        }
    }

    /** The same for WebFlux services: caller tag and the {@code /metrics} alias. */
    @Configuration(proxyBeanMethods = false)
    @ConditionalOnWebApplication(type = ConditionalOnWebApplication.Type.REACTIVE)
    @ConditionalOnClass(name = "org.springframework.boot.actuate.metrics.web.reactive.server.DefaultWebFluxTagsProvider")
    static class ReactiveMetrics {

        @Bean
        @ConditionalOnMissingBean(org.springframework.boot.actuate.metrics.web.reactive.server.WebFluxTagsProvider.class)
        public CallerFluxTagsProvider foremastCallerFluxTags(K8sMetricsProperties props) {
            return new CallerFluxTagsProvider(props.getCallerHeader(), props.getCallerDefault());
        }

        /** {@code GET /metrics} served by the actuator's Prometheus scrape (path rewrite). */
        @Bean
        @ConditionalOnProperty(prefix = "k8s.metrics", name = "metrics-path-alias", matchIfMissing = true)
        public org.springframework.web.server.WebFilter foremastFluxMetricsAlias() {
            return (exchange, chain) -> "/metrics".equals(exchange.getRequest().getPath().value())
                    ? chain.filter(exchange.mutate().request(r -> r.path("/actuator/prometheus")).build())
                    : chain.filter(exchange);
        }
    }
}
